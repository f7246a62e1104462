"""Per-launch-group kernel time from a rocprofv3 kernel trace (csv), per process, to check
bench.py's roofline against the profiler. Groups (the engine's launch
groups, bench.py / TrainEngine.group_times):
  gemm          gemm_x3_kernel, gemm_dma_kernel, gemm_*_kernel, splitk_reduce*, gemm_bf16*
  spmm_max_fwd  max_fwd_kernel, max_fwd_slice_kernel, max_merge_kernel
  spmm_max_bwd  group_pack_kernel, max_bwd_pull_kernel, sum_merge_kernel
  head          head_kernel, head_final_kernel;   adam  adam_*, cast_*
Usage: python scripts/prof_groups.py <rocprof -d dir> [--bench bench.json] [--json out.json]
The process whose pid bench.json names (its "pid") is the headline; the others are the
child processes (sub-configs, drop-in leg)."""
import argparse
import csv
import glob
import json
import os
import re

RULES = [("gemm", r"gemm_|splitk_reduce"), ("spmm_max_fwd", r"max_fwd_kernel|max_fwd_slice_kernel|max_merge_kernel"),
         ("spmm_max_bwd", r"group_pack_kernel|max_bwd_pull_kernel|sum_merge_kernel"),
         ("head", r"head_kernel|head_final_kernel"), ("adam", r"adam_|cast_f32_bf16")]


def group_of(name):
    base = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
    for g, rx in RULES:
        if re.search(rx, base):
            return g
    return "other"


def load(path):
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name") or row.get("KernelName")
            dur = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
            g = out.setdefault(group_of(name), {"ns": 0, "count": 0})
            g["ns"] += dur
            g["count"] += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--bench")
    ap.add_argument("--json")
    a = ap.parse_args()
    pid = None
    bench = None
    if a.bench:
        with open(a.bench) as f:
            bench = json.loads([ln for ln in f if ln.startswith("{")][-1])
        pid = bench.get("pid")
    res = {}
    for p in sorted(glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)):
        m = re.search(r"(\d+)_kernel_trace", os.path.basename(p))
        res[m.group(1) if m else p] = load(p)
    summary = {}
    for proc, groups in res.items():
        tag = "headline" if (pid is not None and proc == str(pid)) else "child"
        print(f"# process {proc} ({tag})")
        summary[proc] = {"role": tag, "groups": {}}
        for g, v in sorted(groups.items(), key=lambda kv: -kv[1]["ns"]):
            avg = v["ns"] / v["count"] / 1e3
            print(f"  {g:14s} {v['count']:7d} launches  {v['ns'] / 1e3:12.1f} us  {avg:9.2f} us/launch")
            summary[proc]["groups"][g] = {"launches": v["count"], "total_us": round(v["ns"] / 1e3, 1),
                                          "us_per_launch": round(avg, 3)}
    if bench is not None and pid is not None and str(pid) in summary:
        # compare PER STEP: a library call can be more than one kernel dispatch (the grouped
        # weight gradients are a partials launch + a combine launch), so per-dispatch
        # averages do not compare with the bench's per-call figures. Steps = head dispatches
        # / 2 (head_kernel + head_final_kernel every step, in every timing graph too).
        rf = bench["roofline"]
        grp = summary[str(pid)]["groups"]
        g = grp.get("gemm")
        if g and "ms_per_step" in rf and grp.get("head"):
            steps = grp["head"]["launches"] / 2
            prof_ms = g["total_us"] / steps / 1e3
            ratio = rf["ms_per_step"] / prof_ms
            prof_tf = rf["flops_per_step"] / (prof_ms * 1e-3) / 1e12
            print(f"# {steps:.0f} steps; gemm {g['launches'] / steps:.0f} dispatches / {rf['launches_per_step']} "
                  f"library calls per step; bench {rf['ms_per_step']} ms/step (graph replay incl. dispatch gaps) vs "
                  f"rocprof {prof_ms:.4f} ms/step: ratio {ratio:.3f}; rocprof -> {prof_tf:.1f} TFLOP/s, "
                  f"frac {prof_tf / rf['peak']:.4f} (bench frac {rf['frac']})")
            summary["check"] = {"steps": steps, "dispatches_per_step": round(g["launches"] / steps, 2),
                                "calls_per_step": rf["launches_per_step"],
                                "bench_ms_per_step": rf["ms_per_step"], "rocprof_ms_per_step": round(prof_ms, 5),
                                "ratio": round(ratio, 4), "rocprof_tflops": round(prof_tf, 2),
                                "rocprof_frac": round(prof_tf / rf["peak"], 4), "bench_frac": rf["frac"]}
    if a.json:
        with open(a.json, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
