"""Binary-tree depth, 4-wide node and leaf counts of a BASELINE scene's BVH (diagnostics)."""
import sys
sys.path[:0] = [".", "ray-traced-stochastic-depth-map_amd"]
from rsd.frame import CONFIGS, FrameConfig, Renderer
from rsd.scenes import make_scene
for name in sys.argv[1:] or ("suntemple_1080p_q",):
    kw, sc = CONFIGS[name]
    r = Renderer(make_scene(sc), FrameConfig(**kw))
    i = r.gscene.info
    print(name, "binary depth", i.max_depth, "wide depth", i.wide_depth, "wide nodes", i.node_count, "leaves", i.leaf_count, "tris", i.triangle_count, "sah", round(i.sah_cost, 1))
