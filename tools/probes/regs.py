"""Per-kernel VGPRs / spills / occupancy of one csrc file (probe helper):
    python tools/probes/regs.py pyabc_amd/csrc/abc_fused.hip [name-substring]"""
import re
import subprocess
import sys


def main():
    src = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else ""
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-Iinclude", "-Ipyabc_amd/csrc", "-c", src, "-o", "/tmp/regs_probe.o",
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    cur = None
    rows = {}
    for ln in r.stderr.splitlines():
        m = re.search(r"remark:\s+(.*?)(?: \[-Rpass|$)", ln)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = t.split(":", 1)[1].strip()
            rows[cur] = {}
        elif cur and ":" in t:
            k, v = t.split(":", 1)
            rows[cur][k.strip()] = v.strip()
    for n, d in rows.items():
        if key and key not in n:
            continue
        print(f"{d.get('VGPRs', '?'):>4} vgpr {d.get('TotalSGPRs', '?'):>4} sgpr lds {d.get('LDS Size [bytes/block]', '?'):>6}  spill {d.get('VGPRs Spill', '?'):>3}  "
              f"occ {d.get('Occupancy [waves/SIMD]', '?'):>2}  {n[:110]}")


if __name__ == "__main__":
    main()
