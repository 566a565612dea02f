"""Print VGPR / LDS / occupancy per kernel of one source file (compile-time,
no GPU):  python tools/kernel_regs.py cf_grad_bpr.hip [name-filter]
(gradient kernels: cf_grad_<model>.hip; draw / apply: cf_kernels.hip)"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "collaborativefilteringusingtensorflow_amd", "csrc")


def main():
    src = os.path.join(CSRC, sys.argv[1] if len(sys.argv) > 1 else "cf_kernels.hip")
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    extra = os.environ.get("CF_EXTRA_FLAGS", "").split()
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only",
           "-munsafe-fp-atomics", "-I" + os.path.join(ROOT, "include"),
           "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/dev/null"] + extra
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    cur, rows = None, []
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": subprocess.run(["c++filt"], input=t.split(":", 1)[1].strip(),
                                          capture_output=True, text=True).stdout.strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        if filt in r["name"]:
            print("%-70s vgpr=%-4s agpr=%-3s lds=%-6s occ=%s scratch=%s" % (
                r["name"][:70], r.get("VGPRs"), r.get("AGPRs"), r.get("LDS Size [bytes/block]"),
                r.get("Occupancy [waves/SIMD]"), r.get("ScratchSize [bytes/lane]")))


if __name__ == "__main__":
    main()
