"""Per-dispatch durations of the standalone LAP sampler (tools/sampler_prof.py under rocprofv3
--kernel-trace) -> CSV rows (dispatch, grid, duration_ns) + a summary line.  The sampler
dispatches are the rle_level launches with B / 4 = 64 workgroups (x 256 threads); the replay
setup's block-sum recompute (245 workgroups) is excluded.

Usage: python tools/sampler_summary.py <rocprof out dir> <out.csv>"""
import csv
import glob
import sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rle_level" not in r["Kernel_Name"]:
            continue
        grid = int(r.get("Grid_Size_X", r.get("Grid_Size", "0")))
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        rows.append((int(r["Start_Timestamp"]), grid, dur))
rows.sort()
sel = [r for r in rows if r[1] == 64 * 256]
assert sel, "no sampler dispatches (grid 64 x 256) in the trace"
warm = sel[10:]  # the first dispatches pay cold instruction / scalar caches
mean = sum(r[2] for r in warm) / len(warm)
srt = sorted(r[2] for r in warm)
with open(sys.argv[2], "w") as f:
    f.write(f"# rocprofv3 --kernel-trace of tools/sampler_prof.py: standalone OP_SAMPLE_GATHER launches, "
            f"B=256 over a 1M-row TD7 Humanoid LAP replay; {len(warm)} dispatches after 10 warm-up ones; "
            f"mean {mean:.0f} ns, median {srt[len(srt) // 2]} ns, min {srt[0]} ns\n")
    f.write("dispatch,grid_threads,duration_ns\n")
    for i, (_, g, d) in enumerate(sel):
        f.write(f"{i},{g},{d}\n")
print(f"sampler dispatches {len(warm)}: mean {mean:.0f} ns median {srt[len(srt) // 2]} ns min {srt[0]} ns")
