// image_equation.cpp -- host compiler of ImageEquation formulas (csrc/image_eq.h) and the
// rsd_image_equation_compile / _release entry points of include/rsd_graph.h.
//
// Grammar (the HLSL expression subset, precedence as in HLSL):
//   expr    := term (('+' | '-') term)*
//   term    := unary (('*' | '/') unary)*
//   unary   := '-' unary | '+' unary | postfix
//   postfix := primary ('.' swizzle)*
//   primary := number | 'I'digit '[' 'xy' ']' | func '(' expr (',' expr)* ')' | '(' expr ')'
// Widths follow HLSL: a scalar promotes to the other operand's width, two vectors of
// different widths truncate to the smaller, the result must be a scalar or a float4.
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>

#include "../../../include/rsd_graph.h"
#include "../image_eq.h"
#include "../rsd_internal.h"

struct rsd_image_program {
    rsd::IeProgram prog;
};

namespace rsd {
namespace {

struct Parser {
    const std::string& s;
    size_t i = 0;
    IeProgram& p;
    int depth = 0, maxDepth = 0;

    [[noreturn]] void fail(const std::string& what) const {
        throw std::invalid_argument("formula '" + s + "': " + what + " at offset " + std::to_string(i));
    }
    void ws() {
        while (i < s.size() && std::isspace((unsigned char)s[i])) ++i;
    }
    bool eat(char c) {
        ws();
        if (i < s.size() && s[i] == c) { ++i; return true; }
        return false;
    }
    void expect(char c) {
        if (!eat(c)) fail(std::string("expected '") + c + "'");
    }
    void emit(uint8_t op, int delta, uint8_t a = 0, uint8_t b = 0, float k = 0.0f) {
        if (p.n >= kIeMaxInstr) fail("formula too long");
        p.code[p.n++] = IeInstr{op, a, b, 0, k};
        depth += delta;
        if (depth > kIeMaxStack) fail("expression nested too deeply");
        if (depth > maxDepth) maxDepth = depth;
    }
    static int binWidth(int a, int b) { return a == 1 ? b : b == 1 ? a : (a < b ? a : b); }

    int expr() {
        int w = term();
        for (;;) {
            if (eat('+')) { w = binWidth(w, term()); emit(IE_ADD, -1); }
            else if (eat('-')) { w = binWidth(w, term()); emit(IE_SUB, -1); }
            else return w;
        }
    }
    int term() {
        int w = unary();
        for (;;) {
            if (eat('*')) { w = binWidth(w, unary()); emit(IE_MUL, -1); }
            else if (eat('/')) { w = binWidth(w, unary()); emit(IE_DIV, -1); }
            else return w;
        }
    }
    int unary() {
        if (eat('-')) { int w = unary(); emit(IE_NEG, 0); return w; }
        if (eat('+')) return unary();
        return postfix();
    }
    int postfix() {
        int w = primary();
        while (eat('.')) {
            ws();
            size_t st = i;
            while (i < s.size() && std::isalpha((unsigned char)s[i])) ++i;
            std::string sw = s.substr(st, i - st);
            if (sw.empty() || sw.size() > 4) fail("bad swizzle");
            const char* sets[2] = {"xyzw", "rgba"};
            int set = std::strchr(sets[0], sw[0]) ? 0 : 1;
            uint8_t lanes[4];
            for (size_t k = 0; k < sw.size(); ++k) {
                const char* q = std::strchr(sets[set], sw[k]);
                if (!q || !*q) fail("bad swizzle '" + sw + "'");
                int lane = (int)(q - sets[set]);
                if (lane >= w) fail("swizzle '" + sw + "' reads past the value's width");
                lanes[k] = (uint8_t)lane;
            }
            for (size_t k = sw.size(); k < 4; ++k) lanes[k] = sw.size() == 1 ? lanes[0] : lanes[0];
            uint8_t packed = (uint8_t)(lanes[0] | lanes[1] << 2 | lanes[2] << 4 | lanes[3] << 6);
            // a scalar's lanes are all equal: .x of a broadcast scalar is the same broadcast
            emit(IE_SWZ, 0, packed);
            w = (int)sw.size();
        }
        return w;
    }
    int primary() {
        ws();
        if (i >= s.size()) fail("unexpected end");
        char c = s[i];
        if (std::isdigit((unsigned char)c) || c == '.') {
            const char* b = s.c_str() + i;
            char* e = nullptr;
            float v = std::strtof(b, &e);
            if (e == b) fail("bad number");
            i += (size_t)(e - b);
            if (i < s.size() && (s[i] == 'f' || s[i] == 'F' || s[i] == 'h' || s[i] == 'H')) ++i;
            emit(IE_CONST, +1, 0, 0, v);
            return 1;
        }
        if (eat('(')) {
            int w = expr();
            expect(')');
            return w;
        }
        if (!std::isalpha((unsigned char)c)) fail(std::string("unexpected '") + c + "'");
        size_t st = i;
        while (i < s.size() && (std::isalnum((unsigned char)s[i]) || s[i] == '_')) ++i;
        std::string id = s.substr(st, i - st);
        if (id.size() == 2 && id[0] == 'I' && id[1] >= '0' && id[1] <= '3') {
            expect('[');
            ws();
            if (s.compare(i, 2, "xy") != 0) fail("textures are indexed by [xy]");
            i += 2;
            expect(']');
            p.texMask |= 1u << (id[1] - '0');
            emit(IE_TEX, +1, (uint8_t)(id[1] - '0'));
            return 4;
        }
        struct Fn { const char* name; int arity; uint8_t op, id; };
        static const Fn fns[] = {
            {"abs", 1, IE_F1, F1_ABS}, {"saturate", 1, IE_F1, F1_SAT}, {"sqrt", 1, IE_F1, F1_SQRT},
            {"floor", 1, IE_F1, F1_FLOOR}, {"ceil", 1, IE_F1, F1_CEIL}, {"frac", 1, IE_F1, F1_FRAC},
            {"exp2", 1, IE_F1, F1_EXP2}, {"log2", 1, IE_F1, F1_LOG2}, {"exp", 1, IE_F1, F1_EXP},
            {"log", 1, IE_F1, F1_LOG}, {"sin", 1, IE_F1, F1_SIN}, {"cos", 1, IE_F1, F1_COS},
            {"rsqrt", 1, IE_F1, F1_RSQRT}, {"sign", 1, IE_F1, F1_SIGN},
            {"min", 2, IE_F2, F2_MIN}, {"max", 2, IE_F2, F2_MAX}, {"pow", 2, IE_F2, F2_POW},
            {"step", 2, IE_F2, F2_STEP}, {"dot", 2, IE_DOT, 0},
            {"lerp", 3, IE_F3, F3_LERP}, {"clamp", 3, IE_F3, F3_CLAMP},
        };
        int ctorN = id == "float" ? 1 : id == "float2" ? 2 : id == "float3" ? 3 : id == "float4" ? 4 : 0;
        const Fn* fn = nullptr;
        for (auto& f : fns)
            if (id == f.name) fn = &f;
        if (!fn && !ctorN) fail("unknown identifier '" + id + "'");
        expect('(');
        int widths[4] = {0, 0, 0, 0}, n = 0;
        do {
            if (n == 4) fail("too many arguments");
            widths[n++] = expr();
        } while (eat(','));
        expect(')');
        if (ctorN) {
            int sum = 0;
            uint8_t packed = 0;
            for (int k = 0; k < n; ++k) {
                sum += widths[k];
                packed |= (uint8_t)((widths[k] - 1) << (2 * k));
            }
            if (!(sum == ctorN || (n == 1 && widths[0] == 1))) fail(id + "(...): argument widths do not add up");
            emit(IE_CTOR, 1 - n, (uint8_t)n, packed);
            return ctorN;
        }
        if (n != fn->arity) fail(id + " takes " + std::to_string(fn->arity) + " arguments");
        int w = widths[0];
        for (int k = 1; k < n; ++k) w = binWidth(w, widths[k]);
        if (fn->op == IE_DOT) {
            if (widths[0] != widths[1] && widths[0] != 1 && widths[1] != 1) fail("dot of different widths");
            emit(IE_DOT, -1, (uint8_t)w);
            return 1;
        }
        emit(fn->op, 1 - n, fn->id);
        return w;
    }
};

}  // namespace

void compile_image_equation(const std::string& formula, IeProgram& p) {
    std::memset(&p, 0, sizeof(p));
    Parser ps{formula, 0, p};
    int w = ps.expr();
    ps.ws();
    if (ps.i != formula.size()) ps.fail("trailing characters");
    if (w != 1 && w != 4) ps.fail("the result must be a scalar or a float4 (float4 result = (FORMULA))");
    p.width = w;
}

}  // namespace rsd

extern "C" rsd_status rsd_image_equation_compile(const char* formula, rsd_image_program** out) {
    if (!formula || !out) {
        rsd::set_error("rsd_image_equation_compile: null argument");
        return RSD_ERR_INVALID_ARG;
    }
    *out = nullptr;
    auto* prog = new (std::nothrow) rsd_image_program;
    if (!prog) return RSD_ERR_OUT_OF_MEMORY;
    try {
        rsd::compile_image_equation(formula, prog->prog);
    } catch (const std::exception& e) {
        delete prog;
        rsd::set_error(e.what());
        return RSD_ERR_INVALID_ARG;
    }
    *out = prog;
    return RSD_OK;
}

extern "C" void rsd_image_equation_release(rsd_image_program* p) { delete p; }

extern "C" rsd_status rsd_image_equation_info(const rsd_image_program* p, uint32_t* instructions, uint32_t* texture_mask) {
    if (!p) {
        rsd::set_error("rsd_image_equation_info: null program");
        return RSD_ERR_INVALID_ARG;
    }
    if (instructions) *instructions = (uint32_t)p->prog.n;
    if (texture_mask) *texture_mask = p->prog.texMask;
    return RSD_OK;
}

namespace rsd {
const IeProgram& image_program(const rsd_image_program* p) { return p->prog; }
}
