"""Mean counter values per launch of one kernel over rocprofv3 --pmc passes (diagnostics):
python tools/pmc_kernel_summary.py <dir with p*/run_counter_collection.csv> <kernel substring> [--json out]"""
import csv
import glob
import json
import statistics
import sys

root, sub = sys.argv[1], sys.argv[2]
vals, durs = {}, []
for path in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    with open(path) as f:
        for row in csv.DictReader(f):
            if sub not in row.get("Kernel_Name", ""):
                continue
            vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
            if "Start_Timestamp" in row and row.get("Counter_Name", "").startswith("SQ_WAVES"):
                durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3)
out = {k: statistics.median(v) for k, v in sorted(vals.items())}
if durs:
    out["duration_us_median"] = statistics.median(durs)
print(json.dumps(out, indent=1))
if "--json" in sys.argv:
    json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
