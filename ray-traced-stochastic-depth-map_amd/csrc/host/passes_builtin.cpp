// passes_builtin.cpp -- the render passes of the SVAO graph that librsd implements, behind
// the RenderPass interface of graph.h:
//
//   GuardBand             GuardBand.cpp:38-64        dict["guardBand"]
//   GBufferRaster         GBufferRaster.cpp:86-230   depth + faceNormalW (rsd_gbuffer_raster),
//                                                    mvec when connected (rsd_motion_vectors_raster)
//   LinearizeDepth        LinearizeDepth.cpp:73-96   rsd_linearize_depth
//   CompressNormals       CompressNormals.cpp:70-96  rsd_compress_normals (viewSpace, 16 bit)
//   StochasticDepthMapRT  StochasticDepthMapRT.cpp   rsd_sd_trace            (the hot path)
//   SVAO                  SVAO.cpp                   rsd_svao_* + a nested "Stochastic Depth"
//                                                    graph holding StochasticDepthMapRT
//
//   CrossBilateralBlur    CrossBilateralBlur.cpp     rsd_cross_bilateral_blur
//   ImageEquation         ImageEquation.cpp          rsd_image_equation_compile / _run
//   Switch                Switch.cpp                 copy of the selected input
//   TemporalAO            TemporalAO.cpp             rsd_temporal_ao (enabled = False: copy)
//   TAA                   TAA.cpp                    rsd_taa
//   AOFlickerMask         AOFlickerMask.cpp          rsd_ao_flicker_mask
//   BinaryDilation        BinaryDilation.cpp         rsd_binary_dilation
//   DeinterleaveTexture   DeinterleaveTexture.cpp    rsd_deinterleave (16 layers of 1/4 x 1/4)
//   InterleaveTexture     InterleaveTexture.cpp      rsd_interleave
//   RayMinMaxLength       RayMinMaxLength.cpp        rsd_ray_min_max_length
//
// Every other pass type of the reference scripts (ToneMapper, ForwardLighting, ...)
// is outside the hot path; it resolves to a stub that declares whatever fields
// the script connects and does no work, so the scripts build and run unchanged.
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "graph.h"
#include "../../../include/rsd_graph.h"

namespace rsd::host {
namespace {

void check(rsd_status st, const char* what) {
    if (st != RSD_OK) throw std::runtime_error(std::string(what) + ": " + rsd_last_error());
}

// Falcor enums arrive from the scripts as their names ('Back', 'StochasticDepth', ...) or as numbers
uint32_t enumProp(const Properties& p, const std::string& key, std::initializer_list<const char*> names,
                  uint32_t def) {
    if (!p.has(key)) return def;
    auto& v = p.items().at(key);
    if (auto s = std::get_if<std::string>(&v)) {
        uint32_t i = 0;
        for (const char* n : names) {
            if (*s == n) return i;
            ++i;
        }
        throw std::runtime_error("property '" + key + "': unknown value '" + *s + "'");
    }
    return (uint32_t)p.getInt(key, def);
}

const std::initializer_list<const char*> kCullNames = {"None", "Front", "Back"};  // RasterizerState::CullMode
uint32_t toRsdCull(uint32_t falcorCull) {  // Falcor None/Front/Back -> RSD_CULL_NONE/FRONT/BACK
    return falcorCull == 0 ? RSD_CULL_NONE : falcorCull == 1 ? RSD_CULL_FRONT : RSD_CULL_BACK;
}
const std::initializer_list<const char*> kDepthModeNames = {"SingleDepth", "DualDepth", "StochasticDepth",
                                                            "Raytraced"};  // VAO/DepthMode.h
const std::initializer_list<const char*> kImplNames = {"Default", "CoverageMask", "ReservoirSampling",
                                                       "KBuffer"};  // StochasticDepthImplementation.h
const std::initializer_list<const char*> kHitOrderNames = {"Canonical", "Traversal", "Wavefront"};  // rsd.h rsd_hit_order
const std::initializer_list<const char*> kNumericsNames = {"Fast", "Exact"};  // rsd.h rsd_numerics
const std::initializer_list<const char*> kAoKernelNames = {"VAO", "HBAO"};    // AOKernel.h -> rsd_ao_kernel

// the SVAO passes' arithmetic when the graph does not set "numerics": RSD_NUMERICS=exact in the
// environment selects the oracle-exact kernels (tests), otherwise the fast default (rsd.h rsd_numerics)
uint32_t defaultNumerics() {
    const char* e = std::getenv("RSD_NUMERICS");
    return (e && std::string(e) == "exact") ? (uint32_t)RSD_NUMERICS_EXACT : (uint32_t)RSD_NUMERICS_FAST;
}

const SceneRef* requireScene(const SceneRef* s, const std::string& who) {
    if (!s || !s->scene) throw std::runtime_error(who + ": no scene set");
    return s;
}

// ------------------------------------------------------------------------------ stubs
class StubPass : public RenderPass {
public:
    explicit StubPass(const Properties& p) { props_ = p; }
    Reflection reflect(const CompileData&) override { return {}; }
    void execute(Context&, const RenderData&) override {}
    bool acceptsAnyField() const override { return true; }
};

// ------------------------------------------------------------------------------ GuardBand
class GuardBandPass : public RenderPass {
public:
    explicit GuardBandPass(const Properties& p) {
        props_ = p;
        guard_ = (int)p.getInt("guardBand", 64);  // GuardBand.h:54
    }
    Reflection reflect(const CompileData&) override { return {}; }
    void execute(Context&, const RenderData& rd) override {
        // GuardBand.cpp:58-63 (the float2 uv bounds are not used by the hot path)
        rd.getDictionary()["guardBand"] = (int64_t)guard_;
    }

private:
    int guard_;
};

// ------------------------------------------------------------------------------ GBufferRaster
class GBufferRasterPass : public RenderPass {
public:
    explicit GBufferRasterPass(const Properties& p) {
        props_ = p;
        // GBufferRaster.cpp:184: cull = forceCullMode ? cull : Back
        const bool force = p.getBool("forceCullMode", false);
        cull_ = force ? toRsdCull(enumProp(p, "cull", kCullNames, 2)) : RSD_CULL_BACK;
    }
    Reflection reflect(const CompileData&) override {
        Reflection r;
        r.addOutput("depth", "Depth buffer (D32 non-linear, R32F here)").format = Format::R32Float;
        r.addOutput("faceNormalW", "Face normal in world space").format = Format::RGBA32Float;
        Field& mv = r.addOutput("mvec", "Motion vector (uv units, RG32F)");
        mv.format = Format::RG32Float;
        mv.optional = true;  // GBuffer.cpp:48: mvec is an optional channel, computed only when read
        return r;
    }
    void setScene(Context&, const SceneRef* s) override {
        scene_ = s;
        hasPrev_ = false;
    }
    void execute(Context& ctx, const RenderData& rd) override {
        if (!scene_) return;  // GBufferRaster.cpp:157 no scene -> outputs stay cleared
        Texture* d = rd["depth"];
        Texture* n = rd["faceNormalW"];
        check(rsd_gbuffer_raster(scene_->scene, &scene_->camera, d->width, d->height, cull_, (float*)d->ptr,
                                 (float*)n->ptr, ctx.stream),
              "GBufferRaster");
        // mvec (GBufferRaster.cpp:62 "Motion vector").  Static scene: the camera's motion between this frame and the previous execute (the
        // first frame's previous camera is its own, Camera::beginFrame).
        const rsd_camera prev = hasPrev_ ? prevCam_ : scene_->camera;
        prevCam_ = scene_->camera;
        hasPrev_ = true;
        Texture* mv = rd["mvec"];
        if (!mv) return;  // nothing reads mvec: no linearize / motion-vector launches, no scratch
        if (mv->format != Format::RG32Float || mv->width != d->width || mv->height != d->height)
            throw Unsupported("GBufferRaster: mvec must be RG32Float at the depth size");
        // background decided on the raw raster depth (the cleared 1.0), not on its linearisation
        check(rsd_motion_vectors_raster(&scene_->camera, &prev, (const float*)d->ptr, d->width, d->height,
                                        (float*)mv->ptr, ctx.stream),
              "GBufferRaster mvec");
    }
    // further channels (posW, normW, ...) feed passes outside the hot path
    bool acceptsAnyField() const override { return true; }

private:
    const SceneRef* scene_ = nullptr;
    uint32_t cull_;
    rsd_camera prevCam_{};
    bool hasPrev_ = false;
};

// ------------------------------------------------------------------------------ LinearizeDepth
class LinearizeDepthPass : public RenderPass {
public:
    explicit LinearizeDepthPass(const Properties& p) {
        props_ = p;
        const std::string fmt = p.getString("depthFormat", "R32Float");
        if (fmt != "R32Float") throw Unsupported("LinearizeDepth: only depthFormat R32Float is implemented");
    }
    Reflection reflect(const CompileData&) override {
        Reflection r;
        r.addInput("depth", "non-linear depth").format = Format::R32Float;
        r.addOutput("linearDepth", "linear view-depth").format = Format::R32Float;
        return r;
    }
    void setScene(Context&, const SceneRef* s) override { scene_ = s; }
    void execute(Context& ctx, const RenderData& rd) override {
        if (!scene_) return;
        Texture* in = rd["depth"];
        Texture* out = rd["linearDepth"];
        if (in->format != Format::R32Float || in->width != out->width || in->height != out->height)
            throw std::runtime_error("LinearizeDepth: input must be R32Float at the output size");
        check(rsd_linearize_depth((const float*)in->ptr, (float*)out->ptr, out->width * out->height,
                                  scene_->camera.nearZ, scene_->camera.farZ, ctx.stream),
              "LinearizeDepth");
    }

private:
    const SceneRef* scene_ = nullptr;
};

// ------------------------------------------------------------------------------ CompressNormals
class CompressNormalsPass : public RenderPass {
public:
    explicit CompressNormalsPass(const Properties& p) {
        props_ = p;
        if (!p.getBool("viewSpace", true) || !p.getBool("use16Bit", true))
            throw Unsupported("CompressNormals: only viewSpace = True, use16Bit = True is implemented");
    }
    Reflection reflect(const CompileData&) override {
        Reflection r;
        r.addInput("normalW", "World Space Normals").format = Format::RGBA32Float;
        r.addOutput("normalOut", "Compressed Normals (Octa mapping)").format = Format::R16Uint;
        return r;
    }
    void setScene(Context&, const SceneRef* s) override { scene_ = s; }
    void execute(Context& ctx, const RenderData& rd) override {
        if (!scene_) return;
        Texture* in = rd["normalW"];
        Texture* out = rd["normalOut"];
        if (in->format != Format::RGBA32Float || in->width != out->width || in->height != out->height)
            throw std::runtime_error("CompressNormals: input must be RGBA32Float at the output size");
        check(rsd_compress_normals((const float*)in->ptr, (uint16_t*)out->ptr, out->width * out->height,
                                   &scene_->camera, ctx.stream),
              "CompressNormals");
    }

private:
    const SceneRef* scene_ = nullptr;
};

// ------------------------------------------------------------------------------ StochasticDepthMapRT
// StochasticDepthMapRT.cpp:135-155 Properties, :190-216 reflect, :231-331 execute.
class StochasticDepthMapRTPass : public RenderPass {
public:
    explicit StochasticDepthMapRTPass(const Properties& p) {
        props_ = p;
        prm_.sample_count = (uint32_t)p.getInt("SampleCount", 4);
        prm_.cull_mode = toRsdCull(enumProp(p, "CullMode", kCullNames, 2));
        prm_.normalize = p.getBool("normalize", true);
        prm_.alpha_test = p.getBool("AlphaTest", true);
        prm_.jitter = p.getBool("Jitter", false);
        prm_.implementation = enumProp(p, "Implementation", kImplNames, 0);
        prm_.alpha = (float)p.getFloat("Alpha", 0.2);
        prm_.ray_interval = p.getBool("RayInterval", true);
        prm_.guard_band = (int32_t)p.getInt("GuardBand", 0);
        prm_.max_count = (uint32_t)p.getInt("MaxCount", 8);
        prm_.use_16bit = p.getBool("Use16Bit", false);
        // librsd extension: "HitOrder" = "Canonical" (default) | "Traversal" | "Wavefront" (rsd.h rsd_hit_order)
        prm_.hit_order = enumProp(p, "HitOrder", kHitOrderNames, 0);
        if (p.getBool("StoreNormals", false))  // StochasticDepthMapRT.cpp:198-203
            throw Unsupported("StochasticDepthMapRT: Storing normals is not supported yet");
        if (p.getBool("useRayPipeline", true) == false)
            throw Unsupported("StochasticDepthMapRT: the raster variant is not part of librsd");
    }
    Reflection reflect(const CompileData&) override {
        const uint32_t N = prm_.sample_count;
        Reflection r;
        r.addInput("linearZ", "non-linear (primary) depth map").format = Format::R32Float;
        auto& st = r.addInput("stencilMask", "(optional) stencil-mask");
        st.format = Format::R8Uint;
        st.optional = true;
        r.addInput("rayMin", "min ray T distance for depth values").optional = true;
        r.addInput("rayMax", "max ray T distance for depth values").optional = true;
        if (N != 1 && N != 2 && N != 4 && N != 8 && N != 16)  // StochasticDepthMapRT.cpp:190 (+ N = 16)
            throw Unsupported("StochasticDepthMapRT: Only 1, 2, 4 and 8 samples are supported (16: librsd extension)");
        if (prm_.use_16bit && N > 4)  // StochasticDepthMapRT.cpp:199
            throw Unsupported("StochasticDepthMapRT: Only 1, 2 and 4 samples are supported");
        auto& o = r.addOutput("stochasticDepth", "stochastic depths in [0,1]");
        // [layer][y][x][min(N,4)]: R32F / RG32F / RGBA32F, or with Use16Bit R16F / RG16F / RGBA16F
        // (StochasticDepthMapRT.cpp:181-198)
        if (prm_.use_16bit) o.format = N == 1 ? Format::R16Float : N == 2 ? Format::RG16Float : Format::RGBA16Float;
        else o.format = N == 1 ? Format::R32Float : N == 2 ? Format::RG32Float : Format::RGBA32Float;
        o.layers = (N + 3) / 4;
        return r;
    }
    void setScene(Context&, const SceneRef* s) override { scene_ = s; }
    void execute(Context& ctx, const RenderData& rd) override {
        if (!scene_) return;  // StochasticDepthMapRT.cpp:233
        Texture* z = rd["linearZ"];
        Texture* sd = rd["stochasticDepth"];
        Texture* rmin = rd["rayMin"];
        Texture* rmax = rd["rayMax"];
        auto& dict = rd.getDictionary();
        auto it = dict.find("SD_CLEAR");
        if (it != dict.end() && std::holds_alternative<bool>(it->second) && std::get<bool>(it->second))
            if (hipMemsetAsync(sd->ptr, 0, sd->bytes(), ctx.stream) != hipSuccess)
                throw std::runtime_error("StochasticDepthMapRT: clear failed");
        check(rsd_sd_trace(scene_->scene, &scene_->camera, &prm_, (const float*)z->ptr, z->width, z->height,
                           rmin ? (const uint32_t*)rmin->ptr : nullptr, rmax ? (const uint32_t*)rmax->ptr : nullptr,
                           (float*)sd->ptr, sd->width, sd->height, nullptr, ctx.stream),
              "StochasticDepthMapRT");
    }
    const rsd_sd_params& params() const { return prm_; }

private:
    const SceneRef* scene_ = nullptr;
    rsd_sd_params prm_{};
};

// ------------------------------------------------------------------------------ SVAO
// SVAO.cpp:73-100 Properties, :117-140 reflect, :143-190 compile (nested SD graph),
// :192-455 execute.  Members the reference sets only from its GUI (SVAO.h:90-126) are
// accepted as extra Properties with the same defaults: stochSamples, stochMaxCount,
// stochGuardBand, stochJitter, rayInterval, cullMode, sampleCount, stochImplementation; and the
// librsd extensions stochHitOrder (rsd_hit_order, passed on as the SD pass's HitOrder) and numerics
// ("Fast" / "Exact", rsd_numerics of the two SVAO passes; default RSD_NUMERICS from the environment, else Fast).
class SVAOPass : public RenderPass {
public:
    explicit SVAOPass(const Properties& p) {
        props_ = p;
        radius_ = (float)p.getFloat("radius", 0.5);      // VAOData.slang:39
        exponent_ = (float)p.getFloat("exponent", 2.0);  // VAOData.slang:40
        thickness_ = (float)p.getFloat("thickness", 0.0);
        primary_ = enumProp(p, "primaryDepthMode", kDepthModeNames, 0);
        secondary_ = enumProp(p, "secondaryDepthMode", kDepthModeNames, 2);
        divisor_ = (uint32_t)p.getInt("stochMapDivisor", 1);
        dualAo_ = p.getBool("dualAO", false);
        alphaTest_ = p.getBool("alphaTest", true);
        samples_ = (uint32_t)p.getInt("stochSamples", 4);
        maxCount_ = (uint32_t)p.getInt("stochMaxCount", 8);
        guardPx_ = (int32_t)p.getInt("stochGuardBand", 512);
        jitter_ = p.getBool("stochJitter", true);
        rayInterval_ = p.getBool("rayInterval", true);
        cull_ = toRsdCull(enumProp(p, "cullMode", kCullNames, 2));
        directions_ = (uint32_t)p.getInt("sampleCount", 8);
        impl_ = enumProp(p, "stochImplementation", kImplNames, 0);
        hitOrder_ = enumProp(p, "stochHitOrder", kHitOrderNames, 0);  // librsd extension (rsd_hit_order)
        rayPipeline_ = p.getBool("rayPipeline", true);  // SVAO.h:101
        numerics_ = enumProp(p, "numerics", kNumericsNames, defaultNumerics());  // librsd extension (rsd_numerics)
        // AO kernel (SVAO::mKernel, a UI dropdown in the reference, SVAO.cpp:615-620; librsd accepts it as a
        // Property).  The UI scales the radius by 1.5 when it switches to HBAO: a graph that selects HBAO
        // gets that scaled radius unless it sets "radius" itself.
        aoKernel_ = enumProp(p, "aoKernel", kAoKernelNames, 0);
        if (aoKernel_ == RSD_AO_KERNEL_HBAO && !p.has("radius")) radius_ *= 1.5f;
    }
    void checkSupported() const {
        if (primary_ > 1) throw Unsupported("SVAO: primaryDepthMode must be SingleDepth or DualDepth");
        if (secondary_ == 3 && (primary_ != 0 || aoKernel_ != 0))
            throw Unsupported("SVAO: the Raytraced secondary mode supports the VAO kernel with SingleDepth only");
        // Common.slang:51-58 holds sample radii for 8, 16 and 32 directions only
        if (directions_ != 8 && directions_ != 16 && directions_ != 32)
            throw Unsupported("SVAO: sampleCount must be 8, 16 or 32");
    }
    void sdSize(uint32_t w, uint32_t h, rsd_vao_data* vao, uint32_t* sw, uint32_t* sh) const {
        // getExtraGuardBand (SVAO.cpp:718-723): only the StochasticDepth mode has an SD guard band
        check(rsd_svao_make_vao_data(w, h, divisor_, secondary_ == 2 ? guardPx_ : 0, radius_, exponent_, thickness_, vao,
                                     sw, sh),
              "SVAO");
    }
    Reflection reflect(const CompileData& cd) override {
        checkSupported();  // reported when the graph is planned, before any device work
        rsd_vao_data vao;
        uint32_t sw = 1, sh = 1;
        if (cd.defaultWidth && cd.defaultHeight) sdSize(cd.defaultWidth, cd.defaultHeight, &vao, &sw, &sh);
        Reflection r;
        auto opt = [&](const char* n, const char* d) { r.addInput(n, d).optional = true; };
        opt("gbufferDepth", "Non-Linear Depth from the G-Buffer");
        r.addInput("depth", "Linear Depth-buffer").format = Format::R32Float;
        opt("depth2", "Linear Depth-buffer of second layer");
        r.addInput("normals", "View space normals, 2x8 octahedral").format = Format::R16Uint;
        opt("color", "Color for pixel importance");
        // SVAO.cpp:129-131: RG8Unorm (bright, dark) with dualAO
        r.addOutput("ao", "Ambient Occlusion (bright/dark if dualAO is enabled)").format =
            dualAo_ ? Format::RG8Unorm : Format::R8Unorm;
        // NUM_DIRECTIONS 8 / 16 / 32 -> R8Uint / R16Uint / R32Uint (SVAO.cpp:132-135)
        r.addOutput("stencil", "Stencil Bitmask for primary / secondary ao").format =
            directions_ > 16 ? Format::R32Uint : directions_ > 8 ? Format::R16Uint : Format::R8Uint;
        for (const char* n : {"internalRayMin", "internalRayMax"}) {
            auto& f = r.addOutput(n, n[8] == 'M' && n[10] == 'n' ? "internal ray min" : "internal ray max");
            f.format = Format::R32Uint;  // R32Int in the reference; the bit patterns are non-negative floats
            f.width = sw;
            f.height = sh;
        }
        return r;
    }
    void setScene(Context& ctx, const SceneRef* s) override {
        scene_ = s;
        if (sdGraph_) sdGraph_->setScene(ctx, s);
    }
    void compile(Context& ctx, const CompileData& cd) override {
        checkSupported();
        width_ = cd.defaultWidth;
        height_ = cd.defaultHeight;
        sdSize(width_, height_, &vao_, &sdW_, &sdH_);
        svp_ = rsd_svao_params{directions_, samples_, secondary_, (uint32_t)rayInterval_, (uint32_t)jitter_, 0,
                               (uint32_t)dualAo_, nullptr, numerics_, aoKernel_, primary_, nullptr};
        sdGraph_.reset();
        if (secondary_ != 2) return;
        // SVAO.cpp:157-189: the nested "Stochastic Depth" graph
        Properties sd;
        sd.set("SampleCount", (int64_t)samples_);
        sd.set("AlphaTest", alphaTest_);
        sd.set("Implementation", (int64_t)impl_);
        sd.set("HitOrder", (int64_t)hitOrder_);
        sd.set("Alpha", (double)(float)(1.5 / samples_));
        sd.set("RayInterval", rayInterval_);
        sd.set("CullMode", std::string(cull_ == RSD_CULL_NONE ? "None" : cull_ == RSD_CULL_FRONT ? "Front" : "Back"));
        sd.set("normalize", true);
        sd.set("StoreNormals", false);
        sd.set("Jitter", jitter_);
        sd.set("GuardBand", (int64_t)vao_.sdGuard);
        sd.set("MaxCount", (int64_t)maxCount_);
        sdGraph_ = std::make_unique<RenderGraph>("Stochastic Depth");
        sdGraph_->createPass("StochasticDepthMap", "StochasticDepthMapRT", sd);
        sdGraph_->markOutput("StochasticDepthMap.stochasticDepth");
        sdGraph_->setScene(ctx, scene_);
        // compiled at the first execute, once its inputs are bound (RenderGraph::execute
        // compiles on demand in the reference, RenderGraph.cpp:420-430)
    }
    void execute(Context& ctx, const RenderData& rd) override {
        if (!scene_) return;  // SVAO.cpp:194
        const SceneRef* s = requireScene(scene_, "SVAO");
        Texture* depth = rd["depth"];
        Texture* normals = rd["normals"];
        Texture* ao = rd["ao"];
        Texture* stencil = rd["stencil"];
        Texture* rmin = rd["internalRayMin"];
        Texture* rmax = rd["internalRayMax"];
        if (depth->width != width_ || depth->height != height_ || normals->width != width_ ||
            normals->height != height_ || depth->format != Format::R32Float || normals->format != Format::R16Uint)
            throw std::runtime_error("SVAO: depth (R32Float) and normals (R16Uint) must match the frame size");
        // SVAO.cpp:326: the guard band comes from the GuardBand pass through the dictionary
        auto& dict = rd.getDictionary();
        int64_t guard = 0;
        if (auto it = dict.find("guardBand"); it != dict.end() && std::holds_alternative<int64_t>(it->second))
            guard = std::get<int64_t>(it->second);
        svp_.guard_band = (uint32_t)guard;
        svp_.tile_flags = nullptr;
        svp_.d_depth2 = nullptr;
        if (primary_ == 1) {  // DualDepth: the second depth layer (SVAO.cpp:201, gDepthTex2)
            Texture* depth2 = rd["depth2"];
            if (!depth2 || depth2->width != width_ || depth2->height != height_ || depth2->format != Format::R32Float)
                throw std::runtime_error("SVAO: primaryDepthMode DualDepth needs 'depth2' (R32Float, the frame size)");
            svp_.d_depth2 = (const float*)depth2->ptr;
        }
        if (secondary_ == 2) {
            // busy 16x16 tiles of this pass's stencil (rsd_svao_params.tile_flags): pass 1 sets, pass 2
            // consumes; sized by the guard band of this frame, zeroed once per allocation
            const uint32_t n = rsd_svao_tile_count(width_, height_, (uint32_t)guard);
            if (n != flagsN_) {
                rsd_svao_tile_flags_release(flags_);  // librsd's generation state of the old buffer
                (void)hipFree(flags_);
                flags_ = nullptr;
                flagsN_ = 0;
                if (n && (hipMalloc(&flags_, n) != hipSuccess || hipMemsetAsync(flags_, 0, n, ctx.stream) != hipSuccess))
                    throw std::runtime_error("SVAO: tile flag allocation failed");
                flagsN_ = n;
            }
            svp_.tile_flags = flags_;
        }
        if (secondary_ == 2)  // SVAO.cpp:330-341
            check(rsd_svao_clear_intervals((uint32_t*)rmin->ptr, (uint32_t*)rmax->ptr, sdW_ * sdH_, ctx.stream),
                  "SVAO clear");
        check(rsd_svao_pass1(&s->camera, &vao_, &svp_, (const float*)depth->ptr, (const uint16_t*)normals->ptr,
                             width_, height_, (uint8_t*)ao->ptr, (uint8_t*)stencil->ptr, (uint32_t*)rmin->ptr,
                             (uint32_t*)rmax->ptr, sdW_, sdH_, ctx.stream),
              "SVAO AO 1");
        if (secondary_ == 0) return;  // SVAO.cpp:355
        if (secondary_ == 1) {  // DualDepth: "AO 2" refines nothing (no calcAO2 branch); it finalizes the AO
            check(rsd_svao_pass2(&s->camera, &vao_, &svp_, (const float*)depth->ptr, (const uint16_t*)normals->ptr,
                                 width_, height_, (const uint8_t*)stencil->ptr, nullptr, 0, 0, (uint8_t*)ao->ptr,
                                 ctx.stream),
                  "SVAO AO 2 (DualDepth)");
            return;
        }
        if (secondary_ == 3) {  // SVAO.cpp:408-455: refine by tracing the scene
            check(rsd_svao_pass2_raytraced(s->scene, &s->camera, &vao_, &svp_, (const float*)depth->ptr,
                                           (const uint16_t*)normals->ptr, width_, height_, (const uint8_t*)stencil->ptr,
                                           (uint8_t*)ao->ptr, cull_, rayPipeline_ ? 1u : 0u, alphaTest_ ? 1u : 0u,
                                           ctx.stream),
                  "SVAO AO 2 (raytraced)");
            return;
        }
        // SVAO.cpp:364-390: the nested graph traces the stochastic depth map
        sdGraph_->setInput("StochasticDepthMap.linearZ", depth);
        sdGraph_->setInput("StochasticDepthMap.rayMin", rmin);
        sdGraph_->setInput("StochasticDepthMap.rayMax", rmax);
        sdGraph_->dictionary()["SD_CLEAR"] = false;
        if (!sdGraph_->isCompiled()) sdGraph_->compile(ctx, sdW_, sdH_);
        sdGraph_->execute(ctx);
        Texture* sd = sdGraph_->getOutput("StochasticDepthMap.stochasticDepth");
        check(rsd_svao_pass2(&s->camera, &vao_, &svp_, (const float*)depth->ptr, (const uint16_t*)normals->ptr,
                             width_, height_, (const uint8_t*)stencil->ptr, (const float*)sd->ptr, sdW_, sdH_,
                             (uint8_t*)ao->ptr, ctx.stream),
              "SVAO AO 2");
    }
    ~SVAOPass() override {
        rsd_svao_tile_flags_release(flags_);
        (void)hipFree(flags_);
    }
    RenderGraph* stochasticDepthGraph() { return sdGraph_.get(); }

private:
    const SceneRef* scene_ = nullptr;
    float radius_, exponent_, thickness_;
    uint32_t primary_, secondary_, divisor_, samples_, maxCount_, cull_, directions_, impl_, hitOrder_, numerics_,
        aoKernel_ = 0;
    int32_t guardPx_;
    bool dualAo_, alphaTest_, jitter_, rayInterval_, rayPipeline_;
    uint32_t width_ = 0, height_ = 0, sdW_ = 0, sdH_ = 0;
    rsd_vao_data vao_{};
    rsd_svao_params svp_{};
    uint8_t* flags_ = nullptr;  // busy-tile flags (rsd_svao_params.tile_flags)
    uint32_t flagsN_ = 0;
    std::unique_ptr<RenderGraph> sdGraph_;
};

// ------------------------------------------------------------------------------ CrossBilateralBlur
// CrossBilateralBlur.cpp:56-149 + CrossBilateralBlur.h:56-66 defaults (enabled, KERNEL_RADIUS 4,
// 1 repetition, betterSlope).  The reference takes no properties (UI only); librsd accepts
// the UI values as optional properties.
class CrossBilateralBlurPass : public RenderPass {
public:
    explicit CrossBilateralBlurPass(const Properties& p) {
        props_ = p;
        enabled_ = p.getBool("enabled", true);
        radius_ = (uint32_t)p.getInt("kernelRadius", 4);
        repetitions_ = (uint32_t)p.getInt("repetitions", 1);
        betterSlope_ = p.getBool("betterSlope", true);
        if (radius_ < 1 || radius_ > 20) throw std::runtime_error("CrossBilateralBlur: kernelRadius must be 1..20");
    }
    ~CrossBilateralBlurPass() override { (void)hipFree(pingpong_); }
    Reflection reflect(const CompileData&) override {
        Reflection r;
        r.addInput("color", "color image to be blurred").format = Format::R8Unorm;
        r.addInput("linear depth", "linear depth").format = Format::R32Float;
        r.addOutput("colorOut", "blurred color").format = Format::R8Unorm;
        return r;
    }
    void compile(Context&, const CompileData& cd) override {
        (void)hipFree(pingpong_);
        pingpong_ = nullptr;
        if (hipMalloc(&pingpong_, (size_t)cd.defaultWidth * cd.defaultHeight) != hipSuccess)
            throw std::runtime_error("CrossBilateralBlur: ping-pong allocation failed");
    }
    void execute(Context& ctx, const RenderData& rd) override {
        Texture* in = rd["color"];
        Texture* z = rd["linear depth"];
        Texture* out = rd["colorOut"];
        if (in->format != Format::R8Unorm || in->width != out->width || in->height != out->height)
            throw Unsupported("CrossBilateralBlur: the color input must be R8Unorm at the output size");
        if (!enabled_) {  // :120-124 blit
            if (hipMemcpyAsync(out->ptr, in->ptr, out->bytes(), hipMemcpyDeviceToDevice, ctx.stream) != hipSuccess)
                throw std::runtime_error("CrossBilateralBlur: copy failed");
            return;
        }
        if (z->format != Format::R32Float) throw Unsupported("CrossBilateralBlur: linear depth must be R32Float");
        auto& dict = rd.getDictionary();
        auto it = dict.find("guardBand");
        const int64_t g = it != dict.end() && std::holds_alternative<int64_t>(it->second)
                              ? std::get<int64_t>(it->second) : 0;
        for (uint32_t k = 0; k < repetitions_; ++k)  // :136-148: every repetition blurs the input again
            check(rsd_cross_bilateral_blur((const uint8_t*)in->ptr, (const float*)z->ptr, z->width, z->height,
                                           (uint8_t*)pingpong_, (uint8_t*)out->ptr, out->width, out->height,
                                           (uint32_t)g, radius_, betterSlope_ ? 1u : 0u, ctx.stream),
                  "CrossBilateralBlur");
    }

private:
    bool enabled_, betterSlope_;
    uint32_t radius_, repetitions_;
    void* pingpong_ = nullptr;
};

// ------------------------------------------------------------------------------ ImageEquation
// ImageEquation.cpp:43-160: `formula` (default "I0[xy]"), `format` (default RGBA32Float).  An
// invalid formula leaves the pass invalid (execute does nothing), as in the reference.
class ImageEquationPass : public RenderPass {
public:
    explicit ImageEquationPass(const Properties& p) {
        props_ = p;
        formula_ = p.getString("formula", "I0[xy]");
        const std::string f = p.getString("format", "RGBA32Float");
        if (f == "RGBA32Float") fmt_ = Format::RGBA32Float;
        else if (f == "RG32Float") fmt_ = Format::RG32Float;
        else if (f == "R32Float") fmt_ = Format::R32Float;
        else if (f == "R8Unorm") fmt_ = Format::R8Unorm;
        else throw Unsupported("ImageEquation: format '" + f + "' (librsd: RGBA32Float, RG32Float, R32Float, R8Unorm)");
        if (rsd_image_equation_compile(formula_.c_str(), &prog_) != RSD_OK) {
            std::fprintf(stderr, "[rsd] ImageEquation: %s\n", rsd_last_error());  // :138-150 logWarning
            prog_ = nullptr;
        }
    }
    ~ImageEquationPass() override { rsd_image_equation_release(prog_); }
    Reflection reflect(const CompileData&) override {
        Reflection r;
        for (const char* n : {"I0", "I1", "I2", "I3"}) r.addInput(n, "input image").optional = true;
        r.addOutput("out", "output image").format = fmt_;
        return r;
    }
    void execute(Context& ctx, const RenderData& rd) override {
        if (!prog_) return;
        rsd_texture in[4] = {};
        const char* names[4] = {"I0", "I1", "I2", "I3"};
        for (int k = 0; k < 4; ++k)
            if (Texture* t = rd[names[k]]) in[k] = rsd_texture{t->ptr, t->width, t->height, t->layers,
                                                                (uint32_t)t->format, (uint64_t)t->bytes()};
        Texture* o = rd["out"];
        rsd_texture out{o->ptr, o->width, o->height, o->layers, (uint32_t)o->format, (uint64_t)o->bytes()};
        check(rsd_image_equation_run(prog_, in, &out, ctx.stream), "ImageEquation");
    }

private:
    std::string formula_;
    Format fmt_;
    rsd_image_program* prog_ = nullptr;
};

// ------------------------------------------------------------------------------ Switch
// Switch.cpp:41-150: inputs i0..i<count-1> (optional), `selected`, output shaped like the
// selected input, blit per execute.
class SwitchPass : public RenderPass {
public:
    explicit SwitchPass(const Properties& p) {
        props_ = p;
        count_ = (int)p.getInt("count", 2);
        selected_ = (int)p.getInt("selected", 0);
        if (count_ < 1 || count_ > 16) throw std::runtime_error("Switch: count must be 1..16");
    }
    Reflection reflect(const CompileData&) override {
        Reflection r;
        for (int k = 0; k < count_; ++k) r.addInput("i" + std::to_string(k), "input").optional = true;
        r.addOutput("out", "selected output").formatFrom = "i" + std::to_string(selected_);
        return r;
    }
    void execute(Context& ctx, const RenderData& rd) override {
        Texture* in = rd["i" + std::to_string(selected_)];
        if (!in) return;  // :141
        Texture* out = rd["out"];
        if (in->bytes() != out->bytes()) throw std::runtime_error("Switch: input and output shapes differ");
        if (hipMemcpyAsync(out->ptr, in->ptr, out->bytes(), hipMemcpyDeviceToDevice, ctx.stream) != hipSuccess)
            throw std::runtime_error("Switch: copy failed");
    }

private:
    int count_, selected_;
};

// ------------------------------------------------------------------------------ TemporalAO
// TemporalAO.cpp:52-169: `enabled` (default True), `useStableMask`.  Disabled: blit aoIn to aoOut
// and drop the history (:128-135, what scripts/SVAO.py configures).  Enabled: rsd_temporal_ao
// against the previous frame's depth / AO / history (allocated on the first enabled frame,
// reset by compile, :105-111, 137-140), then the end-of-frame copies (:165-168).
class TemporalAOPass : public RenderPass {
public:
    explicit TemporalAOPass(const Properties& p) {
        props_ = p;
        enabled_ = p.getBool("enabled", true);
        useStableMask_ = p.getBool("useStableMask", false);
    }
    ~TemporalAOPass() override { release(); }
    Reflection reflect(const CompileData&) override {
        Reflection r;
        r.addInput("aoIn", "AO").format = Format::R8Unorm;
        Field& z = r.addInput("linearZ", "linear depth");
        z.optional = !enabled_;
        z.format = Format::R32Float;
        Field& mv = r.addInput("mvec", "motion vectors");
        mv.optional = !enabled_;
        mv.format = Format::RG32Float;
        r.addInput("stableMask", "stable mask").optional = true;
        r.addOutput("aoOut", "AO").format = Format::R8Unorm;
        return r;
    }
    void compile(Context&, const CompileData&) override { release(); }
    void setScene(Context&, const SceneRef* s) override {
        scene_ = s;
        hasPrev_ = false;
    }
    void execute(Context& ctx, const RenderData& rd) override {
        Texture* in = rd["aoIn"];
        Texture* out = rd["aoOut"];
        if (in->format != Format::R8Unorm || in->bytes() != out->bytes())
            throw std::runtime_error("TemporalAO: aoIn must be R8Unorm at the output size");
        if (!scene_) return;  // :115
        if (!enabled_) {      // :128-135 blit, drop the history
            release();
            if (hipMemcpyAsync(out->ptr, in->ptr, out->bytes(), hipMemcpyDeviceToDevice, ctx.stream) != hipSuccess)
                throw std::runtime_error("TemporalAO: copy failed");
            return;
        }
        Texture* z = rd["linearZ"];
        Texture* mv = rd["mvec"];
        Texture* mask = useStableMask_ ? rd["stableMask"] : nullptr;
        const uint32_t W = out->width, H = out->height;
        if (z->format != Format::R32Float || z->width != W || z->height != H)
            throw Unsupported("TemporalAO: linearZ must be R32Float at the output size");
        if (mv->format != Format::RG32Float || mv->width != W || mv->height != H)
            throw Unsupported("TemporalAO: mvec must be RG32Float at the output size");
        if (mask && (formatBytes(mask->format) != 1 || mask->width != W || mask->height != H))
            throw Unsupported("TemporalAO: stableMask must be an 8-bit mask at the output size");
        if (!prevDepth_ || W != w_ || H != h_) {  // allocatePrevFrameTexture
            release();
            const size_t px = (size_t)W * H;
            if (hipMalloc(&prevDepth_, px * 4) != hipSuccess || hipMalloc(&prevAo_, px) != hipSuccess ||
                hipMalloc(&prevHist_, px) != hipSuccess || hipMalloc(&hist_, px) != hipSuccess) {
                release();
                throw std::runtime_error("TemporalAO: history allocation failed");
            }
            w_ = W;
            h_ = H;
            (void)hipMemsetAsync(prevDepth_, 0, px * 4, ctx.stream);
            (void)hipMemsetAsync(prevAo_, 0, px, ctx.stream);
            (void)hipMemsetAsync(prevHist_, 0, px, ctx.stream);
            (void)hipMemsetAsync(hist_, 0, px, ctx.stream);
        }
        auto& dict = rd.getDictionary();
        auto it = dict.find("guardBand");
        const int64_t g = it != dict.end() && std::holds_alternative<int64_t>(it->second)
                              ? std::get<int64_t>(it->second) : 0;
        // :156 prevViewToCurView = viewMat * inverse(prevViewMat); the view matrix is rigid
        const rsd_camera& cur = scene_->camera;
        const rsd_camera prev = hasPrev_ ? prevCam_ : cur;
        prevCam_ = cur;
        hasPrev_ = true;
        double inv[16] = {};
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) inv[r * 4 + c] = prev.viewMat[c * 4 + r];
            inv[r * 4 + 3] = -((double)prev.viewMat[0 * 4 + r] * prev.viewMat[3] +
                               (double)prev.viewMat[1 * 4 + r] * prev.viewMat[7] +
                               (double)prev.viewMat[2 * 4 + r] * prev.viewMat[11]);
        }
        inv[15] = 1.0;
        float m[16];
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) {
                double acc = 0.0;
                for (int k = 0; k < 4; ++k) acc += (double)cur.viewMat[r * 4 + k] * inv[k * 4 + c];
                m[r * 4 + c] = (float)acc;
            }
        check(rsd_temporal_ao((const uint8_t*)in->ptr, (const float*)z->ptr, (const float*)mv->ptr, prevDepth_,
                              prevAo_, prevHist_, mask ? (const uint8_t*)mask->ptr : nullptr, W, H, (uint32_t)g,
                              &cur, m, (uint8_t*)out->ptr, hist_, ctx.stream),
              "TemporalAO");
        const size_t px = (size_t)W * H;
        if (hipMemcpyAsync(prevDepth_, z->ptr, px * 4, hipMemcpyDeviceToDevice, ctx.stream) != hipSuccess ||
            hipMemcpyAsync(prevAo_, out->ptr, px, hipMemcpyDeviceToDevice, ctx.stream) != hipSuccess ||
            hipMemcpyAsync(prevHist_, hist_, px, hipMemcpyDeviceToDevice, ctx.stream) != hipSuccess)
            throw std::runtime_error("TemporalAO: history copy failed");
    }

private:
    void release() {
        (void)hipFree(prevDepth_);
        (void)hipFree(prevAo_);
        (void)hipFree(prevHist_);
        (void)hipFree(hist_);
        prevDepth_ = nullptr;
        prevAo_ = prevHist_ = hist_ = nullptr;
        w_ = h_ = 0;
    }
    bool enabled_, useStableMask_;
    const SceneRef* scene_ = nullptr;
    rsd_camera prevCam_{};
    bool hasPrev_ = false;
    float* prevDepth_ = nullptr;
    uint8_t *prevAo_ = nullptr, *prevHist_ = nullptr, *hist_ = nullptr;
    uint32_t w_ = 0, h_ = 0;
};

// ------------------------------------------------------------------------------ TAA
// TAA.cpp:59-124: `alpha`, `colorBoxSigma`, `antiFlicker` (TAA.h defaults 0.1, 1.0, true); the
// previous output is kept (allocatePrevColor: re-allocated, zeroed, when the size changes) and
// refreshed by a copy after every execute (:123).
class TAAPass : public RenderPass {
public:
    explicit TAAPass(const Properties& p) {
        props_ = p;
        alpha_ = (float)p.getFloat("alpha", 0.1);
        sigma_ = (float)p.getFloat("colorBoxSigma", 1.0);
        antiFlicker_ = p.getBool("antiFlicker", true);
    }
    ~TAAPass() override { (void)hipFree(prev_); }
    Reflection reflect(const CompileData&) override {
        Reflection r;
        r.addInput("motionVecs", "Screen-space motion vectors").format = Format::RG32Float;
        r.addInput("colorIn", "Color-buffer of the current frame").format = Format::RGBA32Float;
        r.addOutput("colorOut", "Anti-aliased color buffer").format = Format::RGBA32Float;
        return r;
    }
    void execute(Context& ctx, const RenderData& rd) override {
        Texture* in = rd["colorIn"];
        Texture* mv = rd["motionVecs"];
        Texture* out = rd["colorOut"];
        if (in->format != Format::RGBA32Float || in->width != out->width || in->height != out->height)
            throw Unsupported("TAA: colorIn must be RGBA32Float at the output size");
        if (mv->format != Format::RG32Float || mv->width != out->width || mv->height != out->height)
            throw Unsupported("TAA: motionVecs must be RG32Float at the output size");
        if (!prev_ || w_ != out->width || h_ != out->height) {
            (void)hipFree(prev_);
            prev_ = nullptr;
            if (hipMalloc(&prev_, out->bytes()) != hipSuccess) throw std::runtime_error("TAA: history allocation failed");
            (void)hipMemsetAsync(prev_, 0, out->bytes(), ctx.stream);
            w_ = out->width;
            h_ = out->height;
        }
        check(rsd_taa((const float*)in->ptr, (const float*)mv->ptr, (const float*)prev_, out->width, out->height,
                      alpha_, sigma_, antiFlicker_ ? 1u : 0u, (float*)out->ptr, ctx.stream),
              "TAA");
        if (hipMemcpyAsync(prev_, out->ptr, out->bytes(), hipMemcpyDeviceToDevice, ctx.stream) != hipSuccess)
            throw std::runtime_error("TAA: history copy failed");
    }

private:
    float alpha_, sigma_;
    bool antiFlicker_;
    void* prev_ = nullptr;
    uint32_t w_ = 0, h_ = 0;
};

// ------------------------------------------------------------------------------ AOFlickerMask
// AOFlickerMask.cpp:59-86: linearZ + normalW -> R8Uint stable mask (no properties; no scene: no-op)
class AOFlickerMaskPass : public RenderPass {
public:
    explicit AOFlickerMaskPass(const Properties& p) { props_ = p; }
    Reflection reflect(const CompileData&) override {
        Reflection r;
        r.addInput("linearZ", "linear depths").format = Format::R32Float;
        r.addInput("normalW", "world space normals").format = Format::RGBA32Float;
        r.addOutput("mask", "mask with stable pixels (1) and unstable/flickering (0)").format = Format::R8Uint;
        return r;
    }
    void setScene(Context&, const SceneRef* s) override { scene_ = s; }
    void execute(Context& ctx, const RenderData& rd) override {
        if (!scene_) return;
        Texture* z = rd["linearZ"];
        Texture* n = rd["normalW"];
        Texture* m = rd["mask"];
        if (z->format != Format::R32Float || n->format != Format::RGBA32Float || z->width != m->width ||
            z->height != m->height || n->width != m->width || n->height != m->height)
            throw Unsupported("AOFlickerMask: linearZ R32Float and normalW RGBA32Float at the output size");
        check(rsd_ao_flicker_mask((const float*)z->ptr, (const float*)n->ptr, m->width, m->height, &scene_->camera,
                                  (uint8_t*)m->ptr, ctx.stream),
              "AOFlickerMask");
    }

private:
    const SceneRef* scene_ = nullptr;
};

// ------------------------------------------------------------------------------ BinaryDilation
// BinaryDilation.cpp:44-110: `op` = "min" (default) or "max" (the shader's OP define)
class BinaryDilationPass : public RenderPass {
public:
    explicit BinaryDilationPass(const Properties& p) {
        props_ = p;
        const std::string op = p.getString("op", "min");
        if (op != "min" && op != "max") throw Unsupported("BinaryDilation: op must be 'min' or 'max'");
        opMax_ = op == "max";
    }
    Reflection reflect(const CompileData&) override {
        Reflection r;
        r.addInput("input", "binary input").format = Format::R8Uint;
        r.addOutput("output", "dilated binary output").format = Format::R8Uint;
        return r;
    }
    void execute(Context& ctx, const RenderData& rd) override {
        Texture* in = rd["input"];
        Texture* out = rd["output"];
        if (formatBytes(in->format) != 1 || in->width != out->width || in->height != out->height)
            throw Unsupported("BinaryDilation: input must be an 8-bit mask at the output size");
        check(rsd_binary_dilation((const uint8_t*)in->ptr, out->width, out->height, opMax_ ? 1u : 0u,
                                  (uint8_t*)out->ptr, ctx.stream),
              "BinaryDilation");
    }

private:
    bool opMax_;
};

// ------------------------------------------------------------------------------ (De)interleave
// DeinterleaveTexture.cpp:80-158: texIn -> texOut, a 16-layer array of ceil(w/4) x ceil(h/4) in the
// input's format (depth formats arrive as R32Float here).  InterleaveTexture.cpp:62-110: the
// inverse, output in the input's format at the graph's default size.
class DeinterleaveTexturePass : public RenderPass {
public:
    explicit DeinterleaveTexturePass(const Properties& p) { props_ = p; }
    Reflection reflect(const CompileData&) override {
        Reflection r;
        r.addInput("texIn", "texture 2D");
        Field& o = r.addOutput("texOut", "texture 2D array");
        o.formatFrom = "texIn";
        o.shrink = 4;
        o.layersOut = 16;
        return r;
    }
    void execute(Context& ctx, const RenderData& rd) override {
        Texture* in = rd["texIn"];
        Texture* out = rd["texOut"];
        if (in->layers != 1 || out->layers != 16 || out->format != in->format ||
            out->width != (in->width + 3) / 4 || out->height != (in->height + 3) / 4)
            throw Unsupported("DeinterleaveTexture: output must be 16 layers of ceil(w/4) x ceil(h/4) in the input format");
        check(rsd_deinterleave(in->ptr, in->width, in->height, (uint32_t)formatBytes(in->format), out->ptr, ctx.stream),
              "DeinterleaveTexture");
    }
};

class InterleaveTexturePass : public RenderPass {
public:
    explicit InterleaveTexturePass(const Properties& p) { props_ = p; }
    Reflection reflect(const CompileData&) override {
        Reflection r;
        r.addInput("texIn", "Texture2DArray");
        Field& o = r.addOutput("texOut", "Texture2D");
        o.formatFrom = "texIn";
        o.fromFormatOnly = true;
        return r;
    }
    void execute(Context& ctx, const RenderData& rd) override {
        Texture* in = rd["texIn"];
        Texture* out = rd["texOut"];
        if (in->layers == 1) return;  // fed by a stub pass (e.g. ConvolutionalNet): no data to interleave
        if (in->layers != 16 || in->format != out->format || in->width != (out->width + 3) / 4 ||
            in->height != (out->height + 3) / 4)
            throw Unsupported("InterleaveTexture: input must be 16 layers of ceil(w/4) x ceil(h/4) of the output");
        check(rsd_interleave(in->ptr, out->width, out->height, (uint32_t)formatBytes(in->format), out->ptr, ctx.stream),
              "InterleaveTexture");
    }
};

// ------------------------------------------------------------------------------ RayMinMaxLength
// RayMinMaxLength.cpp:55-95: kRayMin + kRayMax (SVAO's internal interval maps) -> len (R32Float,
// the inputs' size)
class RayMinMaxLengthPass : public RenderPass {
public:
    explicit RayMinMaxLengthPass(const Properties& p) { props_ = p; }
    Reflection reflect(const CompileData&) override {
        Reflection r;
        r.addInput("kRayMin", "Minimum ray length");
        r.addInput("kRayMax", "Maximum ray length");
        Field& o = r.addOutput("len", "Ray Length");
        o.format = Format::R32Float;
        o.formatFrom = "kRayMin";
        o.fromSizeOnly = true;
        return r;
    }
    void execute(Context& ctx, const RenderData& rd) override {
        Texture* mn = rd["kRayMin"];
        Texture* mx = rd["kRayMax"];
        Texture* out = rd["len"];
        if (formatBytes(mn->format) != 4 || formatBytes(mx->format) != 4 || mn->width != out->width ||
            mn->height != out->height || mx->width != out->width || mx->height != out->height)
            throw Unsupported("RayMinMaxLength: 32-bit interval maps at the output size");
        check(rsd_ray_min_max_length((const uint32_t*)mn->ptr, (const uint32_t*)mx->ptr, out->width, out->height,
                                     (float*)out->ptr, ctx.stream),
              "RayMinMaxLength");
    }
};

template <class T>
PluginRegistry::Factory factory() {
    return [](const Properties& p) { return std::unique_ptr<RenderPass>(new T(p)); };
}

}  // namespace

void registerBuiltinPasses(PluginRegistry& r) {
    r.registerClass("__Stub", "pass outside the librsd hot path (no work)", factory<StubPass>());
    r.registerClass("GuardBand", "guard band size into the graph dictionary", factory<GuardBandPass>());
    r.registerClass("GBufferRaster", "depth + face normal G-buffer", factory<GBufferRasterPass>());
    r.registerClass("LinearizeDepth", "non-linear -> linear view depth", factory<LinearizeDepthPass>());
    r.registerClass("CompressNormals", "view-space 2x8 octahedral normals", factory<CompressNormalsPass>());
    r.registerClass("StochasticDepthMapRT", "ray-traced stochastic depth map", factory<StochasticDepthMapRTPass>());
    r.registerClass("SVAO", "stochastic-depth volumetric ambient occlusion", factory<SVAOPass>());
    r.registerClass("CrossBilateralBlur", "depth-aware cross bilateral blur", factory<CrossBilateralBlurPass>());
    r.registerClass("ImageEquation", "per-pixel formula over up to 4 images", factory<ImageEquationPass>());
    r.registerClass("Switch", "forwards the selected input", factory<SwitchPass>());
    r.registerClass("TemporalAO", "temporal AO accumulation over motion vectors", factory<TemporalAOPass>());
    r.registerClass("TAA", "temporal anti-aliasing (colour-box clamped history)", factory<TAAPass>());
    r.registerClass("AOFlickerMask", "stable-pixel mask from depth and normals", factory<AOFlickerMaskPass>());
    r.registerClass("BinaryDilation", "min / max over a radius-2 gather ring", factory<BinaryDilationPass>());
    r.registerClass("DeinterleaveTexture", "4x4 deinterleave into 16 quarter-size layers", factory<DeinterleaveTexturePass>());
    r.registerClass("InterleaveTexture", "16 quarter-size layers back into one image", factory<InterleaveTexturePass>());
    r.registerClass("RayMinMaxLength", "SD ray interval lengths (debug view)", factory<RayMinMaxLengthPass>());
}

}  // namespace rsd::host
