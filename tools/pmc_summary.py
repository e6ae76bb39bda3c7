#!/usr/bin/env python3
"""Summary of tools/pmc_pass1.sh's PMC passes for one kernel (diagnostics): per-wave instruction counts
by class, the wave-cycle split (issuing / waiting at s_waitcnt / issue-stalled), the VALU class shares
and the VALU issue utilisation, each counter the median over the kernel's launches.

    python tools/pmc_summary.py gpurun_out/<tag>/pmc_pass1 svao_pass1_kernel [--label "..."] > summary.json

Reads p<i>/run_counter_collection.csv (rocprofv3 --pmc ... --output-format csv) of every pass, and
the kernel-trace durations of the same launches.  The VALU rate is SQ_INSTS_VALU (all waves) x 64 lanes over
the kernel's duration against the nominal issue rate."""
import csv
import json
import statistics
import sys
from collections import defaultdict
from pathlib import Path

d = Path(sys.argv[1])
kern = sys.argv[2]
label = sys.argv[sys.argv.index("--label") + 1] if "--label" in sys.argv else kern
vals = defaultdict(list)
durs = []
for f in sorted(d.glob("p*/run_counter_collection.csv")):
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        key = r["Dispatch_Id"]
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        per[key]["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for key, c in per.items():
        for n, v in c.items():
            if n == "_dur":
                durs.append(v)
            else:
                vals[n].append(v)
med = {n: statistics.median(v) for n, v in vals.items()}
waves = med.get("SQ_WAVES")
if not waves:
    sys.exit("no SQ_WAVES for kernel %r under %s" % (kern, d))
inst = {n: round(v / waves, 1) for n, v in sorted(med.items()) if n.startswith("SQ_INSTS")}
out = {"kernel": label, "launches": len(vals["SQ_WAVES"]), "duration_us": round(statistics.median(durs), 1),
       "waves": waves, "per_wave": inst}
wc = med.get("SQ_WAVE_CYCLES")
if wc:
    out["wave_cycle_split"] = {k: round(med[c] / wc, 3) for k, c in
                               (("active_inst_any", "SQ_ACTIVE_INST_ANY"), ("wait_any_(waitcnt)", "SQ_WAIT_ANY"),
                                ("wait_inst_any_(issue_stall)", "SQ_WAIT_INST_ANY")) if c in med}
valu = med.get("SQ_INSTS_VALU")
if valu:
    classes = [n for n in med if n.startswith("SQ_INSTS_VALU_")]
    share = {n[len("SQ_INSTS_VALU_"):]: round(med[n] / valu, 3) for n in sorted(classes)}
    share["unclassified_(cmp/cndmask/mov/minmax/pk)"] = round(1 - sum(med[n] for n in classes) / valu, 3)
    out["valu_class_share"] = share
if valu:
    # lane-instructions per second over the kernel's duration against the nominal VALU issue rate
    # (1024 SIMDs x 32 lanes per cycle x 2.4 GHz = 78.6 T lane-instr/s, MI355X_MICROARCH.md)
    rate = valu * 64 / (out["duration_us"] * 1e-6)  # valu: the launch's total (all waves)
    out["valu_lane_instr_per_s"] = round(rate / 1e12, 2)
    out["valu_issue_frac_of_peak"] = round(rate / 78.64e12, 3)
print(json.dumps(out, indent=1))
