"""Per-kernel VGPR / AGPR / spill / occupancy from hipcc -Rpass-analysis=kernel-resource-usage.
usage: python tools/resusage.py file.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
inc = ["-I/root/repo/include", "-I/root/repo/matcha-tts-etu-upmc-ensam_amd/csrc"]
out = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", *inc, "-c", src, "-o", "/tmp/_ru.o",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if flt in r["name"]:
        print(f"{r['name'][:90]:90s} V={r.get('VGPRs')} A={r.get('AGPRs')} spill={r.get('VGPRs Spill')} "
              f"occ={r.get('Occupancy [waves/SIMD]')} lds={r.get('LDS Size [bytes/block]')}")
