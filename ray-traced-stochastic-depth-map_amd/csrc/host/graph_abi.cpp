// graph_abi.cpp -- include/rsd_graph.h: the C ABI over the C++ render-graph host.
// Exceptions stop here: each entry point catches, records rsd_last_error() and returns a status.
#include <cstring>

#include "../../../include/rsd_graph.h"
#include "../rsd_internal.h"
#include "graph.h"

using namespace rsd::host;

struct rsd_graph {
    explicit rsd_graph(const char* n) : graph(n ? n : "") {}
    RenderGraph graph;
    SceneRef scene;
    bool hasScene = false;
    std::map<std::string, Texture> inputs;
};

namespace {

template <class F>
rsd_status guarded(const char* who, F&& f) {
    try {
        return f();
    } catch (const Unsupported& e) {
        rsd::set_error(std::string(who) + ": " + e.what());
        return RSD_ERR_UNSUPPORTED;
    } catch (const std::bad_alloc&) {
        rsd::set_error(std::string(who) + ": out of memory");
        return RSD_ERR_OUT_OF_MEMORY;
    } catch (const std::exception& e) {
        rsd::set_error(std::string(who) + ": " + e.what());
        return RSD_ERR_INVALID_ARG;
    }
}

rsd_status nullArg(const char* who) {
    rsd::set_error(std::string(who) + ": null argument");
    return RSD_ERR_INVALID_ARG;
}

rsd_status copyOut(const std::string& s, char* buf, size_t cap, size_t* needed) {
    if (needed) *needed = s.size() + 1;
    if (buf && cap) {
        const size_t n = std::min(cap - 1, s.size());
        std::memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return RSD_OK;
}

Context makeCtx(rsd_graph* g, rsd_stream stream) {
    Context c;
    c.stream = (hipStream_t)stream;
    c.device = g->hasScene && g->scene.scene ? g->scene.scene->dev : nullptr;
    return c;
}

}  // namespace

extern "C" {

rsd_status rsd_graph_create(const char* name, rsd_graph** out) {
    if (!out) return nullArg("rsd_graph_create");
    return guarded("rsd_graph_create", [&] {
        *out = new rsd_graph(name);
        return RSD_OK;
    });
}

void rsd_graph_destroy(rsd_graph* g) { delete g; }

rsd_status rsd_graph_create_pass(rsd_graph* g, const char* pass_name, const char* type, const char* props_json) {
    if (!g || !pass_name || !type) return nullArg("rsd_graph_create_pass");
    return guarded("rsd_graph_create_pass", [&] {
        g->graph.createPass(pass_name, type, Properties::fromJson(props_json ? props_json : "{}"));
        return RSD_OK;
    });
}

rsd_status rsd_graph_add_edge(rsd_graph* g, const char* src, const char* dst) {
    if (!g || !src || !dst) return nullArg("rsd_graph_add_edge");
    return guarded("rsd_graph_add_edge", [&] {
        g->graph.addEdge(src, dst);
        return RSD_OK;
    });
}

rsd_status rsd_graph_mark_output(rsd_graph* g, const char* name) {
    if (!g || !name) return nullArg("rsd_graph_mark_output");
    return guarded("rsd_graph_mark_output", [&] {
        g->graph.markOutput(name);
        return RSD_OK;
    });
}

rsd_status rsd_graph_set_scene(rsd_graph* g, rsd_scene* scene, const rsd_camera* cam) {
    if (!g || !scene || !cam) return nullArg("rsd_graph_set_scene");
    return guarded("rsd_graph_set_scene", [&] {
        const bool changed = !g->hasScene || g->scene.scene != scene;
        g->scene.scene = scene;
        g->scene.camera = *cam;  // passes read the camera through the SceneRef every execute
        g->hasScene = true;
        if (changed) {
            Context c = makeCtx(g, nullptr);
            g->graph.setScene(c, &g->scene);
        }
        return RSD_OK;
    });
}

rsd_status rsd_graph_set_input(rsd_graph* g, const char* name, const rsd_texture* tex) {
    if (!g || !name || !tex || !tex->ptr) return nullArg("rsd_graph_set_input");
    return guarded("rsd_graph_set_input", [&] {
        // every real format of rsd_format (RSD_FMT_UNKNOWN is a graph-internal placeholder)
        if (tex->format > RSD_FMT_RG8UNORM || tex->format == RSD_FMT_UNKNOWN)
            throw std::runtime_error("bad format");
        Texture& t = g->inputs[name];
        t.ptr = tex->ptr;
        t.width = tex->width;
        t.height = tex->height;
        t.layers = tex->layers ? tex->layers : 1;
        t.format = (Format)tex->format;
        g->graph.setInput(name, &t);
        return RSD_OK;
    });
}

rsd_status rsd_graph_compile(rsd_graph* g, uint32_t width, uint32_t height, rsd_stream stream) {
    if (!g) return nullArg("rsd_graph_compile");
    if (!width || !height) {
        rsd::set_error("rsd_graph_compile: empty frame");
        return RSD_ERR_INVALID_ARG;
    }
    return guarded("rsd_graph_compile", [&] {
        Context c = makeCtx(g, stream);
        g->graph.compile(c, width, height);
        return RSD_OK;
    });
}

rsd_status rsd_graph_plan(rsd_graph* g, uint32_t width, uint32_t height) {
    if (!g) return nullArg("rsd_graph_plan");
    if (!width || !height) {
        rsd::set_error("rsd_graph_plan: empty frame");
        return RSD_ERR_INVALID_ARG;
    }
    return guarded("rsd_graph_plan", [&] {
        Context c = makeCtx(g, nullptr);
        g->graph.compile(c, width, height, false);
        return RSD_OK;
    });
}

rsd_status rsd_graph_resources(const rsd_graph* g, char* buf, size_t cap, size_t* needed) {
    if (!g) return nullArg("rsd_graph_resources");
    std::string s;
    for (auto& [k, t] : g->graph.resources())
        s += k + " " + std::to_string(t.width) + " " + std::to_string(t.height) + " " + std::to_string(t.layers) +
             " " + formatName(t.format) + "\n";
    return copyOut(s, buf, cap, needed);
}

rsd_status rsd_graph_execute(rsd_graph* g, rsd_stream stream) {
    if (!g) return nullArg("rsd_graph_execute");
    return guarded("rsd_graph_execute", [&] {
        Context c = makeCtx(g, stream);
        g->graph.execute(c);
        return RSD_OK;
    });
}

rsd_status rsd_graph_get_output(rsd_graph* g, const char* name, rsd_texture* out) {
    if (!g || !name || !out) return nullArg("rsd_graph_get_output");
    Texture* t = g->graph.getOutput(name);
    if (!t) {
        rsd::set_error(std::string("rsd_graph_get_output: '") + name + "' is not a resource of the compiled graph");
        return RSD_ERR_INVALID_ARG;
    }
    *out = rsd_texture{t->ptr, t->width, t->height, t->layers, (uint32_t)t->format, (uint64_t)t->bytes()};
    return RSD_OK;
}

rsd_status rsd_graph_copy_output(rsd_graph* g, const char* name, void* dst, uint64_t bytes, rsd_stream stream) {
    if (!g || !name || !dst) return nullArg("rsd_graph_copy_output");
    Texture* t = g->graph.getOutput(name);
    if (!t || !t->ptr) {
        rsd::set_error(std::string("rsd_graph_copy_output: '") + name + "' is not a resource of the compiled graph");
        return RSD_ERR_INVALID_ARG;
    }
    if (bytes != t->bytes()) {
        rsd::set_error("rsd_graph_copy_output: size mismatch (" + std::to_string(bytes) + " vs " +
                       std::to_string(t->bytes()) + " bytes)");
        return RSD_ERR_INVALID_ARG;
    }
    RSD_HIP(hipMemcpyAsync(dst, t->ptr, bytes, hipMemcpyDefault, (hipStream_t)stream));
    return RSD_OK;
}

rsd_status rsd_graph_execution_order(const rsd_graph* g, char* buf, size_t cap, size_t* needed) {
    if (!g) return nullArg("rsd_graph_execution_order");
    std::string s;
    for (auto& n : g->graph.executionOrder()) s += n + "\n";
    return copyOut(s, buf, cap, needed);
}

rsd_status rsd_graph_pass_times(rsd_graph* g, float* ms, uint32_t cap, uint32_t* count) {
    if (!g || !count) return nullArg("rsd_graph_pass_times");
    return guarded("rsd_graph_pass_times", [&] {
        (void)hipDeviceSynchronize();
        auto t = g->graph.passTimesMs();
        *count = (uint32_t)t.size();
        for (uint32_t i = 0; i < cap && i < t.size() && ms; ++i) ms[i] = t[i].second;
        return RSD_OK;
    });
}

rsd_status rsd_graph_get_dict_int(const rsd_graph* g, const char* key, int64_t* out) {
    if (!g || !key || !out) return nullArg("rsd_graph_get_dict_int");
    auto& d = const_cast<rsd_graph*>(g)->graph.dictionary();
    auto it = d.find(key);
    if (it == d.end() || !std::holds_alternative<int64_t>(it->second)) {
        rsd::set_error(std::string("rsd_graph_get_dict_int: no integer entry '") + key + "'");
        return RSD_ERR_INVALID_ARG;
    }
    *out = std::get<int64_t>(it->second);
    return RSD_OK;
}

rsd_status rsd_graph_pass_count(const rsd_graph* g, uint32_t* passes, uint32_t* edges) {
    if (!g || !passes || !edges) return nullArg("rsd_graph_pass_count");
    *passes = (uint32_t)g->graph.passCount();
    *edges = (uint32_t)g->graph.edgeCount();
    return RSD_OK;
}

rsd_status rsd_plugin_set_dir(const char* dir) {
    if (!dir) return nullArg("rsd_plugin_set_dir");
    PluginRegistry::pluginDir() = dir;
    return RSD_OK;
}

rsd_status rsd_plugin_types(char* buf, size_t cap, size_t* needed) {
    return guarded("rsd_plugin_types", [&] {
        std::string s;
        for (auto& t : PluginRegistry::instance().types())
            if (t != "__Stub") s += t + "\n";
        return copyOut(s, buf, cap, needed);
    });
}

}  // extern "C"
