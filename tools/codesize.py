"""Approximate code bytes of each op-kind / GEMM-variant region of rle_level (from the .s)."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "sac-td3-td7_amd/csrc/kernels.hip"
asm = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-Iinclude",
                      "-Isac-td3-td7_amd/csrc", "-S", "--cuda-device-only", src, "-o", "-"],
                     capture_output=True, text=True).stdout.split("\n")
marks = [(i, l.strip()) for i, l in enumerate(asm) if "; op case" in l or "; gemm variant" in l]
size = lambda ins: 8 if re.search(r"_e64|v_mfma|buffer_|global_|s_load|v_.*(_f64|fma|cndmask_b32_e64|lshl_add|add3|mad)|ds_|s_waitcnt_\w+", ins) else 4
for (i, name), (j, _) in zip(marks, marks[1:] + [(len(asm), "")]):
    body = [l.strip() for l in asm[i + 1:j] if l.strip() and not l.strip().startswith((";", ".")) and not re.match(r"^\S+:", l.strip())]
    print(f"{name[2:60]:60s} {len(body):6d} instrs ~{sum(size(b) for b in body) / 1024:6.1f} KB")
