# The AO chain of the reference's scripts/SVAO.py after the SVAO pass:
# SVAO.ao -> CrossBilateralBlur -> TemporalAO (disabled) -> Switch -> ImageEquation, plus
# the R8Unorm / R32Float ImageEquation formulas of scripts/SAVO_record.py.
from falcor import *

def render_graph_svao_post():
    g = RenderGraph('SVAOPost')
    g.create_pass('GuardBand', 'GuardBand', {'guardBand': 16})
    g.create_pass('GBufferRaster', 'GBufferRaster', {'outputSize': 'Default', 'samplePattern': 'Center', 'forceCullMode': False, 'cull': 'Back'})
    g.create_pass('LinearizeDepth', 'LinearizeDepth', {'depthFormat': 'R32Float'})
    g.create_pass('CompressNormals', 'CompressNormals', {'viewSpace': True, 'use16Bit': True})
    g.create_pass('SVAO', 'SVAO', {'radius': 1.0, 'primaryDepthMode': 'SingleDepth', 'secondaryDepthMode': 'StochasticDepth', 'exponent': 2.0, 'thickness': 0.0, 'stochMapDivisor': 2, 'dualAO': False, 'alphaTest': True, 'stochGuardBand': 64})
    g.create_pass('CrossBilateralBlur0', 'CrossBilateralBlur', {})
    g.create_pass('TemporalAO', 'TemporalAO', {'enabled': False, 'useStableMask': True})
    g.create_pass('AOSwitch', 'Switch', {'count': 2, 'selected': 1, 'i0': 'Default', 'i1': 'TemporalAO'})
    g.create_pass('AmbientRef', 'ImageEquation', {'formula': 'I0[xy].rrra', 'format': 'RGBA32Float'})
    g.create_pass('ImageEquation1', 'ImageEquation', {'formula': '1.0 - max(I0[xy].x-I0[xy].y, 0.05)', 'format': 'R8Unorm'})
    g.create_pass('ImageEquationLinearDepth', 'ImageEquation', {'formula': 'I0[xy]/1000.0', 'format': 'R32Float'})
    g.add_edge('GuardBand', 'GBufferRaster')
    g.add_edge('GBufferRaster.depth', 'LinearizeDepth.depth')
    g.add_edge('GBufferRaster.depth', 'SVAO.gbufferDepth')
    g.add_edge('GBufferRaster.faceNormalW', 'CompressNormals.normalW')
    g.add_edge('LinearizeDepth.linearDepth', 'SVAO.depth')
    g.add_edge('CompressNormals.normalOut', 'SVAO.normals')
    g.add_edge('SVAO.ao', 'CrossBilateralBlur0.color')
    g.add_edge('LinearizeDepth.linearDepth', 'CrossBilateralBlur0.linear depth')
    g.add_edge('CrossBilateralBlur0.colorOut', 'TemporalAO.aoIn')
    g.add_edge('LinearizeDepth.linearDepth', 'TemporalAO.linearZ')
    g.add_edge('GBufferRaster.mvec', 'TemporalAO.mvec')
    g.add_edge('CrossBilateralBlur0.colorOut', 'AOSwitch.i0')
    g.add_edge('TemporalAO.aoOut', 'AOSwitch.i1')
    g.add_edge('AOSwitch.out', 'AmbientRef.I0')
    g.add_edge('AmbientRef.out', 'ImageEquation1.I0')
    g.add_edge('LinearizeDepth.linearDepth', 'ImageEquationLinearDepth.I0')
    g.mark_output('AmbientRef.out')
    g.mark_output('ImageEquation1.out')
    g.mark_output('ImageEquationLinearDepth.out')
    return g

SVAOPost = render_graph_svao_post()
try: m.addGraph(SVAOPost)
except NameError: None
