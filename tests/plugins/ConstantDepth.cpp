// A render-pass plugin built outside librsd (tests/test_graph.py): it is found by the
// registry as <plugin dir>/ConstantDepth.so and registered through the extern "C"
// registerPlugin entry, the loading protocol of Falcor's Plugin.cpp:56-91.
#include "graph.h"

namespace {
using namespace rsd::host;

class ConstantDepth : public RenderPass {
public:
    explicit ConstantDepth(const Properties& p) { value_ = (float)p.getFloat("value", 1.0); }
    Reflection reflect(const CompileData&) override {
        Reflection r;
        r.addOutput("depth", "constant R32F image").format = Format::R32Float;
        return r;
    }
    void execute(Context&, const RenderData&) override {}

private:
    float value_;
};
}  // namespace

extern "C" void registerPlugin(PluginRegistry& r) {
    r.registerClass("ConstantDepth", "constant depth image",
                    [](const Properties& p) { return std::unique_ptr<RenderPass>(new ConstantDepth(p)); });
}
