"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin): one line per kernel."""
import re
import sys

cur = None
rows = {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
pat = sys.argv[1] if len(sys.argv) > 1 else ""
for k, v in rows.items():
    if pat in k:
        print(k[-60:], "VGPR", v.get("VGPRs"), "AGPR", v.get("AGPRs"), "spill", v.get("VGPRs Spill"),
              "scratch", v.get("ScratchSize [bytes/lane]"), "occ", v.get("Occupancy [waves/SIMD]"))
