"""Summarise -Rpass-analysis=kernel-resource-usage remarks per kernel."""
import re
import sys

cur = None
rows = {}
for line in open(sys.argv[1]):
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+?): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    if any(x in k for x in ("k_scan", "k_eval", "k_detect", "k_stream", "k_collect")):
        print("%-50s VGPR %3s spillV %4s scratch %5s occ %s LDS %s" % (
            k[:50], v.get("VGPRs"), v.get("VGPRs Spill"), v.get("ScratchSize [bytes/lane]"),
            v.get("Occupancy [waves/SIMD]"), v.get("LDS Size [bytes/block]")))
