"""Copy one GPU round's outputs (tools/gpu_round.sh <tag>, tools/profile_dl_trace.sh <tag>) from
gpurun_out/ into profiles/ and record its PMC summary in profiles/pmc_traffic.json.

    python tools/collect_round.py <tag>
"""
import json
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
tag = sys.argv[1]
G, P = ROOT / "gpurun_out", ROOT / "profiles"


def bench_line(log):
    lines = [ln for ln in log.read_text().splitlines() if ln.startswith("{")]
    return lines[-1] + "\n" if lines else None


copies = {
    G / f"prof_{tag}" / "trace_kernel_stats.csv": P / f"{tag}_rocprof_kernel_stats.csv",
    G / f"prof_dl_{tag}" / "trace_kernel_stats.csv": P / f"{tag}_dl_rocprof_kernel_stats.csv",
    G / f"{tag}_pmc_summary.txt": P / f"{tag}_pmc_summary.txt",
    G / f"{tag}_smoke.log": P / f"{tag}_smoke.log",
    G / f"{tag}_long.log": P / f"{tag}_long_bench.txt",
    G / f"{tag}_rate.log": P / f"{tag}_screen_rate.txt",
}
for src, dst in copies.items():
    if src.exists():
        shutil.copy(src, dst)
        print("copied", dst.name)
for src, dst in ((G / f"{tag}_bench.log", P / f"{tag}_bench_default.json"),
                 (G / f"prof_{tag}" / "bench.log", P / f"{tag}_bench_under_rocprof.json"),
                 (G / f"prof_dl_{tag}" / "bench.log", P / f"{tag}_bench_dl_under_rocprof.json")):
    if src.exists() and bench_line(src):
        dst.write_text(bench_line(src))
        print("wrote", dst.name)
tests = G / f"{tag}_gpu_tests.log"
if tests.exists():
    (P / f"{tag}_gpu_tests_tail.txt").write_text("\n".join(tests.read_text().splitlines()[-25:]) + "\n")
    print("wrote", f"{tag}_gpu_tests_tail.txt")
if (G / f"pmc_{tag}").exists():
    subprocess.check_call([sys.executable, str(ROOT / "tools" / "pmc_summary.py"), str(G / f"pmc_{tag}"), "1000000",
                           "--write", "scl_L8_N128_K64_B1000000"])
