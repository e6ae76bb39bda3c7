// graph.h -- the C++ render-graph host of librsd: a MI355X-native restatement of the
// Falcor plugin / RenderPass / RenderGraph surface that the hot-path passes live behind.
//
//   Falcor                                         here
//   Core/Plugin.cpp:45-91  PluginManager +         PluginRegistry: built-in types + dlopen of
//     dlopen(plugins/<T>.so) + registerPlugin        plugins/<Type>.so, extern "C" registerPlugin
//   RenderGraph/RenderPass.h:119-259 virtuals      RenderPass: reflect / compile / setScene / execute
//   Utils/Properties.h:92 Properties               Properties (flat JSON object from the scripts)
//   RenderGraph.cpp:101,249,525,420 createPass /   RenderGraph: createPass / addEdge / markOutput /
//     addEdge / markOutput / execute                 setInput / compile / execute / getOutput
//   RenderGraphCompiler.cpp:48-172 cull + topo     RenderGraph::compile (same culling rule)
//   RenderGraphExe.cpp:33-44 serial execute with   RenderGraph::execute: passes in topological order
//     one FALCOR_PROFILE per pass                    on one HIP stream, one hipEvent pair per pass
//
// Errors are C++ exceptions (std::runtime_error) inside the host, as in Falcor; the C ABI
// of the graph (include/rsd_graph.h) converts them to status codes.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <variant>
#include <vector>

#include "../../../include/rsd.h"

namespace rsd::host {

// a configuration the reference supports but librsd does not (-> RSD_ERR_UNSUPPORTED)
struct Unsupported : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// ---- Properties (Falcor Properties.h:92): the dict a graph script passes to create_pass
class Properties {
public:
    using Value = std::variant<bool, int64_t, double, std::string>;
    static Properties fromJson(const std::string& json);
    bool has(const std::string& k) const { return m_.count(k) != 0; }
    const std::map<std::string, Value>& items() const { return m_; }
    void set(const std::string& k, Value v) { m_[k] = std::move(v); }
    bool getBool(const std::string& k, bool def) const;
    int64_t getInt(const std::string& k, int64_t def) const;
    double getFloat(const std::string& k, double def) const;
    std::string getString(const std::string& k, const std::string& def) const;
    std::string toJson() const;

private:
    std::map<std::string, Value> m_;
};

// ---- resources
enum class Format { R32Float, RG32Float, RGBA32Float, R16Uint, R8Uint, R8Unorm, R32Uint, Unknown,
                    R16Float, RG16Float, RGBA16Float, RG8Unorm };
size_t formatBytes(Format f);
const char* formatName(Format f);

struct Texture {
    void* ptr = nullptr;
    uint32_t width = 0, height = 0, layers = 1;
    Format format = Format::Unknown;
    size_t bytes() const { return (size_t)width * height * layers * formatBytes(format); }
};

struct Field {
    std::string name, desc;
    bool isInput = true;
    bool optional = false;  // input: may stay unconnected; output: allocated only when consumed
    Format format = Format::Unknown;  // Unknown: take it from the connected producer
    uint32_t width = 0, height = 0;  // 0: the graph's default dims
    uint32_t layers = 1;
    std::string formatFrom;  // output: copy format and size from this input's producer (Switch)
    // with formatFrom: divide the copied size by this (rounding up) and set the layer count
    // (DeinterleaveTexture: 4, 16 layers); fromFormatOnly: copy the format only (InterleaveTexture)
    uint32_t shrink = 1, layersOut = 0;
    bool fromFormatOnly = false;
    bool fromSizeOnly = false;  // with formatFrom: copy the size, keep the declared format (RayMinMaxLength)
};

struct Reflection {
    std::vector<Field> fields;
    Field& addInput(const std::string& n, const std::string& d) { fields.push_back({n, d, true}); return fields.back(); }
    Field& addOutput(const std::string& n, const std::string& d) { fields.push_back({n, d, false}); return fields.back(); }
    const Field* find(const std::string& n) const {
        for (auto& f : fields) if (f.name == n) return &f;
        return nullptr;
    }
};

struct CompileData {
    uint32_t defaultWidth = 0, defaultHeight = 0;
};

// The frame's scene: the uploaded BVH and the camera (Falcor Scene + Camera subset).
struct SceneRef {
    rsd_scene* scene = nullptr;
    rsd_camera camera{};
};

using Dictionary = std::map<std::string, Properties::Value>;

struct Context {
    hipStream_t stream = nullptr;
    rsd_device* device = nullptr;
};

class RenderData {
public:
    RenderData(std::map<std::string, Texture*> res, Dictionary& dict, uint32_t w, uint32_t h)
        : res_(std::move(res)), dict_(dict), w_(w), h_(h) {}
    Texture* operator[](const std::string& field) const {
        auto it = res_.find(field);
        return it == res_.end() ? nullptr : it->second;
    }
    Dictionary& getDictionary() const { return dict_; }
    uint32_t defaultWidth() const { return w_; }
    uint32_t defaultHeight() const { return h_; }

private:
    std::map<std::string, Texture*> res_;
    Dictionary& dict_;
    uint32_t w_, h_;
};

class RenderPass {
public:
    virtual ~RenderPass() = default;
    virtual Properties getProperties() const { return props_; }
    virtual Reflection reflect(const CompileData& cd) = 0;
    virtual void compile(Context&, const CompileData&) {}
    virtual void setScene(Context&, const SceneRef*) {}
    virtual void execute(Context& ctx, const RenderData& rd) = 0;
    // stubs accept any field name (pass types outside the hot path)
    virtual bool acceptsAnyField() const { return false; }
    std::string type, name;

protected:
    Properties props_;
};

// ---- plugins (Plugin.cpp:45-91 / Plugin.h:288-323)
class PluginRegistry {
public:
    using Factory = std::function<std::unique_ptr<RenderPass>(const Properties&)>;
    static PluginRegistry& instance();
    void registerClass(const std::string& type, const std::string& desc, Factory f);
    // built-in type, or dlopen("<plugin dir>/<type>.so") + registerPlugin; unknown types
    // become stub passes (logged) so that whole graph scripts load unchanged
    std::unique_ptr<RenderPass> create(const std::string& type, const Properties& props);
    bool isRegistered(const std::string& type) const { return factories_.count(type) != 0; }
    bool loadPlugin(const std::string& type);
    static std::string& pluginDir();
    std::vector<std::string> types() const;

private:
    std::map<std::string, std::pair<std::string, Factory>> factories_;
    std::vector<void*> handles_;
};

// ---- graph (RenderGraph.cpp / RenderGraphCompiler.cpp / RenderGraphExe.cpp)
class RenderGraph {
public:
    explicit RenderGraph(std::string name) : name_(std::move(name)) {}
    ~RenderGraph();
    RenderPass* createPass(const std::string& name, const std::string& type, const Properties& props);
    RenderPass* addPass(std::unique_ptr<RenderPass> pass, const std::string& name);
    void addEdge(const std::string& src, const std::string& dst);  // "pass.field" or "pass"
    void markOutput(const std::string& name);
    void setInput(const std::string& name, Texture* tex);  // external resource bound to pass.field
    void setScene(Context& ctx, const SceneRef* scene);
    // allocate = false plans only (culling, order, resource table) -- no device calls
    void compile(Context& ctx, uint32_t width, uint32_t height, bool allocate = true);
    bool isCompiled() const { return compiled_; }
    void execute(Context& ctx);
    Texture* getOutput(const std::string& name);
    Dictionary& dictionary() { return dict_; }
    const std::string& name() const { return name_; }
    std::vector<std::string> executionOrder() const;
    std::vector<std::pair<std::string, Texture>> resources() const;  // "pass.field" -> texture
    std::vector<std::pair<std::string, float>> passTimesMs() const;  // of the last execute
    size_t passCount() const { return passes_.size(); }
    size_t edgeCount() const { return edges_.size(); }
    RenderPass* getPass(const std::string& name);

private:
    struct Edge { std::string srcPass, srcField, dstPass, dstField; };
    struct PassNode {
        std::unique_ptr<RenderPass> pass;
        Reflection refl;
    };
    void release();
    std::string name_;
    std::map<std::string, PassNode> passes_;
    std::vector<std::string> insertion_;
    std::vector<Edge> edges_;
    std::vector<std::string> outputs_;
    std::map<std::string, Texture*> inputs_;     // "pass.field" -> external texture
    std::map<std::string, Texture> owned_;       // "pass.field" (producer side) -> allocation
    std::map<std::string, std::map<std::string, Texture*>> bindings_;  // pass -> field -> texture
    std::vector<std::string> order_;
    Dictionary dict_;
    const SceneRef* scene_ = nullptr;
    uint32_t width_ = 0, height_ = 0;
    bool compiled_ = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events_;
};

// built-in passes (passes_builtin.cpp)
void registerBuiltinPasses(PluginRegistry& r);

}  // namespace rsd::host
