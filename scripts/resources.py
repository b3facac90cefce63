"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output: name, VGPRs, spills."""
import re
import sys

cur = None
rows = []
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("vspill", r"VGPRs Spill: (\d+)"),
                     ("sspill", r"SGPRs Spill: (\d+)")):
        m = re.search(pat, line)
        if m:
            cur[key] = int(m.group(1))
only_spills = "--spills" in sys.argv
filt = [a for a in sys.argv[2:] if not a.startswith("--")]
for r in rows:
    n = r["name"].replace("_ZN2dl12_GLOBAL__N_1", "")
    if filt and not any(f in n for f in filt):
        continue
    if only_spills and not r.get("vspill"):
        continue
    print(f"{n:70s} vgpr={r.get('vgpr')} spill={r.get('vspill')}")
