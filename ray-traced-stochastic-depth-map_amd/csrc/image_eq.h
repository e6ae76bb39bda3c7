// image_eq.h -- ImageEquation formulas compiled to a small stack program.
//
// Reference: ImageEquation (RenderPasses/ImageEquation/ImageEquation.cpp:134-160) pastes the
// `formula` property into `float4 result = (FORMULA);` of a full-screen pixel shader
// (ImageEquation.ps.slang:8-13) with inputs Texture2D<float4> I0..I3 and `int2 xy` = the
// pixel.  librsd parses the HLSL expression subset the graph scripts use (I<k>[xy],
// swizzles, + - * /, unary -, literals, float2/3/4(...), abs/saturate/sqrt/floor/ceil/frac/
// exp/exp2/log/log2/sin/cos/rsqrt/sign, min/max/pow/step/dot, lerp/clamp) on the host
// (host/image_equation.cpp) into this program; post.hip interprets it per pixel.  Values are
// float4 lanes; a scalar is kept broadcast in all four lanes, which is HLSL's scalar ->
// vector promotion.  All literals are float (HLSL integer division is not modelled).
#pragma once
#include <stdint.h>

namespace rsd {

enum IeOp : uint8_t {
    IE_TEX,    // push I<a>[xy] as float4 (0 when unbound or outside the texture)
    IE_CONST,  // push k broadcast
    IE_SWZ,    // top = top.<a: 4 x 2-bit lane indices>
    IE_ADD, IE_SUB, IE_MUL, IE_DIV,
    IE_NEG,
    IE_F1,     // unary function a (IeF1)
    IE_F2,     // binary function a (IeF2)
    IE_F3,     // ternary function a (IeF3)
    IE_DOT,    // dot over the first a lanes, broadcast
    IE_CTOR,   // floatN(args): a = argument count, b = 4 x 2-bit (width - 1) of the arguments
};
enum IeF1 : uint8_t { F1_ABS, F1_SAT, F1_SQRT, F1_FLOOR, F1_CEIL, F1_FRAC, F1_EXP2, F1_LOG2, F1_EXP, F1_LOG,
                      F1_SIN, F1_COS, F1_RSQRT, F1_SIGN };
enum IeF2 : uint8_t { F2_MIN, F2_MAX, F2_POW, F2_STEP };
enum IeF3 : uint8_t { F3_LERP, F3_CLAMP };

struct IeInstr {
    uint8_t op, a, b, c;
    float k;
};

constexpr int kIeMaxInstr = 64;
constexpr int kIeMaxStack = 8;

struct IeProgram {
    IeInstr code[kIeMaxInstr];
    int32_t n;        // instructions
    int32_t width;    // result width (1 = broadcast scalar, or 4)
    uint32_t texMask; // bit k: the formula reads I<k>
};

}  // namespace rsd
