# The hot-path slice of an SVAO render graph, written in the scripting style the
# reference's graph scripts use (falcor RenderGraph API).  Loaded by tests/test_graph.py
# with rsd.graph.load_script (not executed) and by `import falcor` users as code.
from falcor import *

def render_graph_svao_hotpath():
    g = RenderGraph('SVAOHotPath')
    g.create_pass('GuardBand', 'GuardBand', {'guardBand': 16})
    g.create_pass('GBufferRaster', 'GBufferRaster', {'outputSize': 'Default', 'samplePattern': 'Center', 'forceCullMode': False, 'cull': 'Back'})
    g.create_pass('LinearizeDepth', 'LinearizeDepth', {'depthFormat': 'R32Float'})
    g.create_pass('CompressNormals', 'CompressNormals', {'viewSpace': True, 'use16Bit': True})
    g.create_pass('SVAO', 'SVAO', {'radius': 1.0, 'primaryDepthMode': 'SingleDepth', 'secondaryDepthMode': 'StochasticDepth', 'exponent': 2.0, 'thickness': 0.0, 'stochMapDivisor': 2, 'dualAO': False, 'alphaTest': True, 'stochGuardBand': 64})
    g.create_pass('Blur', 'CrossBilateralBlur', {})
    g.create_pass('Unused', 'ToneMapper', {'operator': 'Linear'})
    g.add_edge('GuardBand', 'GBufferRaster')
    g.add_edge('GBufferRaster.depth', 'LinearizeDepth.depth')
    g.add_edge('GBufferRaster.depth', 'SVAO.gbufferDepth')
    g.add_edge('GBufferRaster.faceNormalW', 'CompressNormals.normalW')
    g.add_edge('LinearizeDepth.linearDepth', 'SVAO.depth')
    g.add_edge('CompressNormals.normalOut', 'SVAO.normals')
    g.add_edge('SVAO.ao', 'Blur.color')
    g.add_edge('LinearizeDepth.linearDepth', 'Blur.linear depth')
    g.mark_output('Blur.colorOut')
    g.mark_output('SVAO.ao')
    return g

SVAOHotPath = render_graph_svao_hotpath()
try: m.addGraph(SVAOHotPath)
except NameError: None
