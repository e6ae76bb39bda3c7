"""Keep the counters of a candidate list that `rocprofv3 -L` (saved to a file) knows, so one missing
counter name does not fail a --pmc pass: python tools/pmc_filter.py <list-file> CTR [CTR ...]
Prints the kept counters space-separated (all of them if the list file is empty or missing)."""
import re
import sys

path, cands = sys.argv[1], sys.argv[2:]
try:
    text = open(path).read()
except OSError:
    text = ""
if not text.strip():
    print(" ".join(cands))
else:
    names = set(re.findall(r"\b([A-Z][A-Z0-9_]+)\b", text))
    print(" ".join(c for c in cands if re.sub(r"_(sum|avr|min|max)$", "", c) in names or c in names))
