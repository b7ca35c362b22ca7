"""Compact per-kernel resource usage of one .hip file (VGPRs, AGPRs, occupancy, scratch, LDS):
python tools/kres.py kge_rel.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c",
                      "knowledge-graph-embedding_amd/csrc/" + src, "-o", "/tmp/kres.o",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for name, r in rows.items():
    if flt in name:
        print("%-70s V%-4s A%-3s occ %-2s scr %-4s lds %s" % (name[:70], r.get("VGPRs"), r.get("AGPRs"),
              r.get("Occupancy [waves/SIMD]"), r.get("ScratchSize [bytes/lane]"), r.get("LDS Size [bytes/block]")))
