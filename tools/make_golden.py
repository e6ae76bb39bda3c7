#!/usr/bin/env python3
"""Generate tests/golden/reference_tables.json from the reference's own files.

Runs ONLY in the build container (it reads /root/reference, which does not exist
on the GPU box); the JSON it writes is committed and is what the tests read.

What it extracts (data only -- inputs and expected values, no source text):
  * jitterPos[16]          StochasticDepthMapRT/Jitter.slangh:20
  * sampleRadius VAO/HBAO  SVAO/Common.slang:51-68 (tables for 8/16/32 directions)
  * GenPoints output       SVAO/GenPoints.py:1-31, executed as a subprocess (32-dir tables)
  * Bayer dither values    SVAO.cpp:670-674 -> R8Unorm bytes as SVAO.cpp:684 computes them
  * VAOData defaults       SVAO/VAOData.slang:35-45
  * SVAO / SD defaults     SVAO.h:90-126, StochasticDepthMapRT.h:62-82
  * the SVAO graph-script properties  scripts/SVAO.py:12
"""
import json
import re
import subprocess
import sys
from pathlib import Path

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parents[1] / "tests" / "golden" / "reference_tables.json"


def floats(text):
    return [float(x) for x in re.findall(r"[-+]?\d*\.\d+(?:[eE][-+]?\d+)?|[-+]?\d+\.(?:[eE][-+]?\d+)?", text)]


def main():
    rp = REF / "Source" / "RenderPasses"
    jit = (rp / "StochasticDepthMapRT" / "Jitter.slangh").read_text().splitlines()
    line = [l for l in jit if l.startswith("static const float2 jitterPos[16]")][0]
    jv = floats(line.split("=", 1)[1])
    assert len(jv) == 32
    jitter = [jv[i:i + 2] for i in range(0, 32, 2)]

    common = (rp / "SVAO" / "Common.slang").read_text().splitlines()
    radius = {"VAO": {}, "HBAO": {}}
    kernel = None
    for l in common:
        if l.startswith("#if AO_KERNEL == AO_KERNEL_VAO"):
            kernel = "VAO"
        elif l.startswith("#if AO_KERNEL == AO_KERNEL_HBAO"):
            kernel = "HBAO"
        m = re.match(r"\s*static const float sampleRadius\[(\d+)\]\s*=\s*\{(.*)\};", l)
        if m and kernel:
            radius[kernel][m.group(1)] = floats(m.group(2))

    gp = subprocess.run([sys.executable, str(rp / "SVAO" / "GenPoints.py")], capture_output=True, text=True, check=True)
    out = gp.stdout.splitlines()
    genpoints = {
        "vdc_32": floats(out[0]),
        "vao_32": floats(out[1].split("[", 1)[1]),
        "hbao_32": floats(out[2].split("[", 1)[1]),
    }

    svao_cpp = (rp / "SVAO" / "SVAO.cpp").read_text()
    dm = re.search(r"const float ditherValues\[\] = \{(.*?)\};", svao_cpp, re.S)
    dither = floats(dm.group(1))
    assert len(dither) == 16

    vd = (rp / "SVAO" / "VAOData.slang").read_text()
    vao_defaults = {}
    for name in ["radius", "exponent", "thickness", "ssRadiusCutoff", "ssMaxRadius"]:
        m = re.search(r"float %s = ([-0-9.]+)f;" % name, vd)
        vao_defaults[name] = float(m.group(1))
    vao_defaults["sdGuard"] = int(re.search(r"int sdGuard = (\d+);", vd).group(1))

    svao_h = (rp / "SVAO" / "SVAO.h").read_text()
    sd_h = (rp / "StochasticDepthMapRT" / "StochasticDepthMapRT.h").read_text()

    def grab(text, pat, conv=int):
        return conv(re.search(pat, text).group(1))

    svao_defaults = {
        "mStochSamples": grab(svao_h, r"uint mStochSamples = (\d+);"),
        "mStochMapDivisor": grab(svao_h, r"uint mStochMapDivisor = (\d+);"),
        "mSampleCount": grab(svao_h, r"uint32_t mSampleCount = (\d+);"),
        "mStochMapGuardBand": grab(svao_h, r"int mStochMapGuardBand = (\d+);"),
        "mStochMaxCount": grab(svao_h, r"int mStochMaxCount = (\d+);"),
        "mStochMapJitter": grab(svao_h, r"bool mStochMapJitter = (\w+);", str) == "true",
        "mUseRayInterval": grab(svao_h, r"bool mUseRayInterval = (\w+);", str) == "true",
    }
    sd_defaults = {
        "mSampleCount": grab(sd_h, r"uint32_t mSampleCount = (\d+);"),
        "mMaxCount": grab(sd_h, r"int mMaxCount = (\d+);"),
        "mGuardBand": grab(sd_h, r"int mGuardBand = (\d+);"),
        "mAlpha": grab(sd_h, r"float mAlpha = ([0-9.]+)f;", float),
        "mNormalize": grab(sd_h, r"bool mNormalize = (\w+);", str) == "true",
        "mJitter": grab(sd_h, r"bool mJitter = (\w+);", str) == "true",
        "mUseRayInterval": grab(sd_h, r"bool mUseRayInterval = (\w+);", str) == "true",
    }

    script = (REF / "scripts" / "SVAO.py").read_text()
    m = re.search(r"g\.create_pass\('SVAO', 'SVAO', (\{.*?\})\)", script)
    svao_script_props = eval(m.group(1), {"__builtins__": {}}, {"True": True, "False": False})  # a dict literal
    m = re.search(r"g\.create_pass\('GuardBand', 'GuardBand', (\{.*?\})\)", script)
    guard_props = eval(m.group(1), {"__builtins__": {}}, {})

    data = {
        "_source": "extracted from /root/reference by tools/make_golden.py",
        "jitterPos": jitter,
        "sampleRadius": radius,
        "genpoints": genpoints,
        "ditherValues": dither,
        "noiseBytes": [int(v / 16.0 * 255.0) for v in dither],
        "vaoDataDefaults": vao_defaults,
        "svaoDefaults": svao_defaults,
        "sdDefaults": sd_defaults,
        "svaoScriptProps": svao_script_props,
        "guardBandScriptProps": guard_props,
    }
    OUT.parent.mkdir(parents=True, exist_ok=True)
    OUT.write_text(json.dumps(data, indent=1) + "\n")
    print("wrote", OUT)


if __name__ == "__main__":
    main()
