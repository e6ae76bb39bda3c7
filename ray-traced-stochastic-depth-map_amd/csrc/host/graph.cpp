// graph.cpp -- Properties, PluginRegistry and RenderGraph of the librsd host (see graph.h).
#include "graph.h"

#include <dlfcn.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <deque>
#include <set>
#include <sstream>

namespace rsd::host {

// ------------------------------------------------------------------------------ Properties
namespace {
struct JsonReader {
    const std::string& s;
    size_t i = 0;
    explicit JsonReader(const std::string& str) : s(str) {}
    void ws() { while (i < s.size() && std::isspace((unsigned char)s[i])) ++i; }
    [[noreturn]] void fail(const char* what) {
        throw std::runtime_error(std::string("Properties JSON: ") + what + " at offset " + std::to_string(i));
    }
    void expect(char c) {
        ws();
        if (i >= s.size() || s[i] != c) fail("unexpected character");
        ++i;
    }
    std::string str() {
        expect('"');
        std::string out;
        while (i < s.size() && s[i] != '"') {
            if (s[i] == '\\' && i + 1 < s.size()) {
                char e = s[++i];
                out += e == 'n' ? '\n' : e == 't' ? '\t' : e;
            } else {
                out += s[i];
            }
            ++i;
        }
        if (i >= s.size()) fail("unterminated string");
        ++i;
        return out;
    }
    Properties::Value value() {
        ws();
        if (i >= s.size()) fail("missing value");
        if (s[i] == '"') return str();
        if (s.compare(i, 4, "true") == 0) { i += 4; return true; }
        if (s.compare(i, 5, "false") == 0) { i += 5; return false; }
        if (s.compare(i, 4, "null") == 0) { i += 4; return std::string(); }
        size_t j = i;
        bool isFloat = false;
        while (j < s.size() && (std::isdigit((unsigned char)s[j]) || s[j] == '-' || s[j] == '+' || s[j] == '.' ||
                                s[j] == 'e' || s[j] == 'E')) {
            if (s[j] == '.' || s[j] == 'e' || s[j] == 'E') isFloat = true;
            ++j;
        }
        if (j == i) fail("unsupported value (flat objects of bool / number / string only)");
        std::string num = s.substr(i, j - i);
        i = j;
        if (isFloat) return std::stod(num);
        return (int64_t)std::stoll(num);
    }
};
}  // namespace

Properties Properties::fromJson(const std::string& json) {
    Properties p;
    JsonReader r(json);
    r.ws();
    if (r.i >= json.size()) return p;
    r.expect('{');
    r.ws();
    if (r.i < json.size() && json[r.i] == '}') return p;
    while (true) {
        std::string k = r.str();
        r.expect(':');
        p.m_[k] = r.value();
        r.ws();
        if (r.i < json.size() && json[r.i] == ',') { ++r.i; continue; }
        r.expect('}');
        break;
    }
    return p;
}

bool Properties::getBool(const std::string& k, bool def) const {
    auto it = m_.find(k);
    if (it == m_.end()) return def;
    if (auto b = std::get_if<bool>(&it->second)) return *b;
    if (auto i = std::get_if<int64_t>(&it->second)) return *i != 0;
    throw std::runtime_error("property '" + k + "' is not a bool");
}
int64_t Properties::getInt(const std::string& k, int64_t def) const {
    auto it = m_.find(k);
    if (it == m_.end()) return def;
    if (auto i = std::get_if<int64_t>(&it->second)) return *i;
    if (auto d = std::get_if<double>(&it->second)) return (int64_t)*d;
    if (auto b = std::get_if<bool>(&it->second)) return *b;
    throw std::runtime_error("property '" + k + "' is not a number");
}
double Properties::getFloat(const std::string& k, double def) const {
    auto it = m_.find(k);
    if (it == m_.end()) return def;
    if (auto d = std::get_if<double>(&it->second)) return *d;
    if (auto i = std::get_if<int64_t>(&it->second)) return (double)*i;
    throw std::runtime_error("property '" + k + "' is not a number");
}
std::string Properties::getString(const std::string& k, const std::string& def) const {
    auto it = m_.find(k);
    if (it == m_.end()) return def;
    if (auto s = std::get_if<std::string>(&it->second)) return *s;
    throw std::runtime_error("property '" + k + "' is not a string");
}
std::string Properties::toJson() const {
    std::ostringstream o;
    o << "{";
    bool first = true;
    for (auto& [k, v] : m_) {
        if (!first) o << ", ";
        first = false;
        o << "\"" << k << "\": ";
        if (auto b = std::get_if<bool>(&v)) o << (*b ? "true" : "false");
        else if (auto i = std::get_if<int64_t>(&v)) o << *i;
        else if (auto d = std::get_if<double>(&v)) { o.precision(17); o << *d; }
        else o << "\"" << std::get<std::string>(v) << "\"";
    }
    o << "}";
    return o.str();
}

size_t formatBytes(Format f) {
    switch (f) {
        case Format::R32Float: case Format::R32Uint: return 4;
        case Format::RG32Float: return 8;
        case Format::RGBA32Float: return 16;
        case Format::R16Uint: case Format::R16Float: case Format::RG8Unorm: return 2;
        case Format::RG16Float: return 4;
        case Format::RGBA16Float: return 8;
        case Format::R8Uint: case Format::R8Unorm: return 1;
        default: return 16;
    }
}
const char* formatName(Format f) {
    switch (f) {
        case Format::R32Float: return "R32Float";
        case Format::RG32Float: return "RG32Float";
        case Format::RGBA32Float: return "RGBA32Float";
        case Format::R16Uint: return "R16Uint";
        case Format::R8Uint: return "R8Uint";
        case Format::R8Unorm: return "R8Unorm";
        case Format::R32Uint: return "R32Uint";
        case Format::R16Float: return "R16Float";
        case Format::RG16Float: return "RG16Float";
        case Format::RGBA16Float: return "RGBA16Float";
        case Format::RG8Unorm: return "RG8Unorm";
        default: return "Unknown";
    }
}

// ------------------------------------------------------------------------------ registry
PluginRegistry& PluginRegistry::instance() {
    static PluginRegistry* r = [] {
        auto* reg = new PluginRegistry();
        registerBuiltinPasses(*reg);
        return reg;
    }();
    return *r;
}

std::string& PluginRegistry::pluginDir() {
    static std::string dir;
    return dir;
}

void PluginRegistry::registerClass(const std::string& type, const std::string& desc, Factory f) {
    factories_[type] = {desc, std::move(f)};
}

bool PluginRegistry::loadPlugin(const std::string& type) {
    if (pluginDir().empty()) return false;
    const std::string path = pluginDir() + "/" + type + ".so";
    void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL);
    if (!h) return false;
    using RegFn = void (*)(PluginRegistry&);
    auto fn = reinterpret_cast<RegFn>(dlsym(h, "registerPlugin"));
    if (!fn) {
        dlclose(h);
        throw std::runtime_error("plugin '" + path + "' has no registerPlugin symbol");
    }
    fn(*this);
    handles_.push_back(h);
    return isRegistered(type);
}

std::vector<std::string> PluginRegistry::types() const {
    std::vector<std::string> t;
    for (auto& [k, v] : factories_) t.push_back(k);
    return t;
}

std::unique_ptr<RenderPass> PluginRegistry::create(const std::string& type, const Properties& props) {
    if (!isRegistered(type)) loadPlugin(type);
    auto it = factories_.find(type);
    std::unique_ptr<RenderPass> p;
    if (it != factories_.end()) p = it->second.second(props);
    else p = factories_.at("__Stub").second(props);  // not on the hot path: no-op pass of that type
    p->type = type;
    return p;
}

// ------------------------------------------------------------------------------ graph
RenderGraph::~RenderGraph() { release(); }

void RenderGraph::release() {
    for (auto& [k, t] : owned_)
        if (t.ptr) (void)hipFree(t.ptr);
    owned_.clear();
    for (auto& e : events_) {
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    events_.clear();
    compiled_ = false;
}

RenderPass* RenderGraph::addPass(std::unique_ptr<RenderPass> pass, const std::string& name) {
    if (passes_.count(name)) throw std::runtime_error("RenderGraph '" + name_ + "': pass '" + name + "' exists");
    pass->name = name;
    RenderPass* raw = pass.get();
    passes_[name].pass = std::move(pass);
    insertion_.push_back(name);
    compiled_ = false;
    return raw;
}

RenderPass* RenderGraph::createPass(const std::string& name, const std::string& type, const Properties& props) {
    return addPass(PluginRegistry::instance().create(type, props), name);
}

RenderPass* RenderGraph::getPass(const std::string& name) {
    auto it = passes_.find(name);
    return it == passes_.end() ? nullptr : it->second.pass.get();
}

static std::pair<std::string, std::string> splitName(const std::string& n) {
    auto d = n.find('.');
    if (d == std::string::npos) return {n, ""};
    return {n.substr(0, d), n.substr(d + 1)};
}

void RenderGraph::addEdge(const std::string& src, const std::string& dst) {
    auto [sp, sf] = splitName(src);
    auto [dp, df] = splitName(dst);
    if (!passes_.count(sp)) throw std::runtime_error("addEdge: unknown pass '" + sp + "'");
    if (!passes_.count(dp)) throw std::runtime_error("addEdge: unknown pass '" + dp + "'");
    if (sf.empty() != df.empty()) throw std::runtime_error("addEdge: data edges connect pass.field to pass.field");
    edges_.push_back({sp, sf, dp, df});
    compiled_ = false;
}

void RenderGraph::markOutput(const std::string& name) {
    auto [p, f] = splitName(name);
    if (!passes_.count(p) || f.empty()) throw std::runtime_error("markOutput: '" + name + "' is not pass.field");
    if (std::find(outputs_.begin(), outputs_.end(), name) == outputs_.end()) outputs_.push_back(name);
    compiled_ = false;
}

void RenderGraph::setInput(const std::string& name, Texture* tex) {
    // rebinding an input of a compiled graph takes effect at the next execute (no recompile),
    // as SVAO.cpp:366-371 rebinds the nested graph's inputs every frame
    const bool known = inputs_.count(name) != 0;
    inputs_[name] = tex;
    if (!known) compiled_ = false;
}

void RenderGraph::setScene(Context& ctx, const SceneRef* scene) {
    scene_ = scene;
    for (auto& [n, node] : passes_) node.pass->setScene(ctx, scene);
}

void RenderGraph::compile(Context& ctx, uint32_t width, uint32_t height, bool allocate) {
    release();
    width_ = width;
    height_ = height;
    CompileData cd{width, height};
    for (auto& [n, node] : passes_) node.refl = node.pass->reflect(cd);

    // RenderGraphCompiler.cpp:121-172: keep the passes that feed a marked output
    std::set<std::string> need;
    std::deque<std::string> q;
    if (outputs_.empty()) for (auto& n : insertion_) q.push_back(n);
    for (auto& o : outputs_) q.push_back(splitName(o).first);
    while (!q.empty()) {
        std::string p = q.front();
        q.pop_front();
        if (!need.insert(p).second) continue;
        for (auto& e : edges_) if (e.dstPass == p) q.push_back(e.srcPass);
    }
    // topological order (Kahn), ties broken by creation order
    std::map<std::string, int> indeg;
    for (auto& p : need) indeg[p] = 0;
    for (auto& e : edges_)
        if (need.count(e.srcPass) && need.count(e.dstPass)) indeg[e.dstPass]++;
    order_.clear();
    std::set<std::string> done;
    while (order_.size() < need.size()) {
        bool progressed = false;
        for (auto& n : insertion_) {
            if (!need.count(n) || done.count(n) || indeg[n] != 0) continue;
            order_.push_back(n);
            done.insert(n);
            for (auto& e : edges_)
                if (e.srcPass == n && need.count(e.dstPass)) indeg[e.dstPass]--;
            progressed = true;
            break;
        }
        if (!progressed) throw std::runtime_error("RenderGraph '" + name_ + "': cycle");
    }

    // resources: every output field of a needed pass (declared, or referenced by an edge
    // or a marked output for stub passes) gets an allocation
    bindings_.clear();
    auto fieldOf = [&](const std::string& p, const std::string& f) -> const Field* {
        return passes_.at(p).refl.find(f);
    };
    std::map<std::string, Field> outs;  // "pass.field" -> field description
    // optional outputs (Falcor RenderPassReflection Field::Flags::Optional) get a resource only when
    // something reads them: an edge into a needed pass or a marked graph output
    std::set<std::string> consumed(outputs_.begin(), outputs_.end());
    for (auto& e : edges_)
        if (!e.srcField.empty() && need.count(e.srcPass) && need.count(e.dstPass))
            consumed.insert(e.srcPass + "." + e.srcField);
    for (auto& p : order_) {
        for (auto& f : passes_.at(p).refl.fields)
            if (!f.isInput && (!f.optional || consumed.count(p + "." + f.name))) outs[p + "." + f.name] = f;
    }
    auto stubOut = [&](const std::string& p, const std::string& f, Format hint) {
        const std::string key = p + "." + f;
        if (outs.count(key)) return;
        if (!passes_.at(p).pass->acceptsAnyField())
            throw std::runtime_error("RenderGraph '" + name_ + "': pass '" + p + "' has no output '" + f + "'");
        Field fd;
        fd.name = f;
        fd.isInput = false;
        fd.format = hint == Format::Unknown ? Format::RGBA32Float : hint;
        outs[key] = fd;
    };
    for (auto& e : edges_) {
        if (e.srcField.empty() || !need.count(e.srcPass) || !need.count(e.dstPass)) continue;
        const Field* in = fieldOf(e.dstPass, e.dstField);
        if (!in && !passes_.at(e.dstPass).pass->acceptsAnyField())
            throw std::runtime_error("RenderGraph '" + name_ + "': pass '" + e.dstPass + "' has no input '" +
                                     e.dstField + "'");
        stubOut(e.srcPass, e.srcField, in ? in->format : Format::Unknown);
    }
    for (auto& o : outputs_) {
        auto [p, f] = splitName(o);
        stubOut(p, f, Format::Unknown);
    }
    // outputs shaped like one of the pass's inputs (Switch.cpp:95-108), in topological order
    for (auto& p : order_) {
        for (auto& [key, f] : outs) {
            if (f.formatFrom.empty() || splitName(key).first != p) continue;
            const Format declared = f.format;
            for (auto& e : edges_) {
                if (e.dstPass != p || e.dstField != f.formatFrom || !need.count(e.srcPass)) continue;
                auto src = outs.find(e.srcPass + "." + e.srcField);
                if (src == outs.end()) continue;
                f.format = src->second.format;
                f.width = src->second.width;
                f.height = src->second.height;
                f.layers = src->second.layers;
            }
            auto ext = inputs_.find(p + "." + f.formatFrom);
            if (ext != inputs_.end() && ext->second) {
                f.format = ext->second->format;
                f.width = ext->second->width;
                f.height = ext->second->height;
                f.layers = ext->second->layers;
            }
            if (f.fromSizeOnly) {
                f.format = declared;
                f.layers = 1;
            } else if (f.fromFormatOnly) {
                f.width = f.height = 0;
                f.layers = 1;
            } else if (f.shrink > 1 || f.layersOut) {
                const uint32_t w = f.width ? f.width : width, h = f.height ? f.height : height;
                f.width = (w + f.shrink - 1) / f.shrink;
                f.height = (h + f.shrink - 1) / f.shrink;
                if (f.layersOut) f.layers = f.layersOut;
            }
        }
    }
    for (auto& [key, f] : outs) {
        Texture t;
        t.width = f.width ? f.width : width_;
        t.height = f.height ? f.height : height_;
        t.layers = f.layers;
        t.format = f.format == Format::Unknown ? Format::RGBA32Float : f.format;
        if (allocate) {
            hipError_t err = hipMalloc(&t.ptr, t.bytes());
            if (err == hipSuccess) err = hipMemsetAsync(t.ptr, 0, t.bytes(), ctx.stream);
            if (err != hipSuccess) {
                (void)hipFree(t.ptr);
                throw std::runtime_error(std::string("RenderGraph allocation: ") + hipGetErrorString(err));
            }
        }
        owned_[key] = t;
        auto [p, fn] = splitName(key);
        bindings_[p][fn] = &owned_[key];
    }
    for (auto& e : edges_) {
        if (e.srcField.empty() || !need.count(e.srcPass) || !need.count(e.dstPass)) continue;
        bindings_[e.dstPass][e.dstField] = &owned_.at(e.srcPass + "." + e.srcField);
    }
    for (auto& [key, tex] : inputs_) {
        auto [p, f] = splitName(key);
        if (need.count(p)) bindings_[p][f] = tex;
    }
    for (auto& p : order_) {
        for (auto& f : passes_.at(p).refl.fields)
            if (f.isInput && !f.optional && !bindings_[p].count(f.name))
                throw std::runtime_error("RenderGraph '" + name_ + "': required input '" + p + "." + f.name +
                                         "' is not connected");
        if (allocate) passes_.at(p).pass->compile(ctx, cd);
    }
    if (!allocate) return;  // plan only: order + resource table, no device work
    events_.resize(order_.size());
    for (auto& e : events_) {
        (void)hipEventCreate(&e.first);
        (void)hipEventCreate(&e.second);
    }
    compiled_ = true;
}

void RenderGraph::execute(Context& ctx) {
    if (!compiled_) throw std::runtime_error("RenderGraph '" + name_ + "': execute before compile");
    for (auto& [key, tex] : inputs_) {
        auto [p, f] = splitName(key);
        auto b = bindings_.find(p);
        if (b != bindings_.end()) b->second[f] = tex;
    }
    for (size_t i = 0; i < order_.size(); ++i) {
        const std::string& p = order_[i];
        RenderData rd(bindings_[p], dict_, width_, height_);
        (void)hipEventRecord(events_[i].first, ctx.stream);
        passes_.at(p).pass->execute(ctx, rd);  // RenderGraphExe.cpp:33-44
        (void)hipEventRecord(events_[i].second, ctx.stream);
    }
}

Texture* RenderGraph::getOutput(const std::string& name) {
    auto it = owned_.find(name);
    return it == owned_.end() ? nullptr : &it->second;
}

std::vector<std::string> RenderGraph::executionOrder() const { return order_; }

std::vector<std::pair<std::string, Texture>> RenderGraph::resources() const {
    return std::vector<std::pair<std::string, Texture>>(owned_.begin(), owned_.end());
}

std::vector<std::pair<std::string, float>> RenderGraph::passTimesMs() const {
    std::vector<std::pair<std::string, float>> t;
    for (size_t i = 0; i < order_.size() && i < events_.size(); ++i) {
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, events_[i].first, events_[i].second) != hipSuccess) ms = -1.0f;
        t.push_back({order_[i], ms});
    }
    return t;
}

}  // namespace rsd::host
