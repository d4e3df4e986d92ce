"""Forensics for a run-to-run difference of the race check: runs one bench layout twice (same settings, by default
DP2 with every side stream folded) with SCALING_AMD_BENCH_TRACE, then reports the first step and quantity where the
two runs differ per rank: the loss (forward of that step), the reduced gradients (backward + DP reduction) or a
parameter (optimizer update).

    python tools/race_trace.py [bench args ...]      (default: --gpus 2)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASE = ["--model", "llama_tiny", "--backend", "gloo-gpu", "--seq-len", "256", "--micro-batch", "2", "--steps", "3",
        "--warmup", "1"]


def run(args, prefix, env_extra):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.update(env_extra)
    env["SCALING_AMD_BENCH_TRACE"] = prefix
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *BASE, *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        print(r.stderr[-3000:])
        raise SystemExit(1)


def load(prefix, rank):
    with open(f"{prefix}.rank{rank}.jsonl") as f:
        return [json.loads(x) for x in f]


def main():
    args = sys.argv[1:] or ["--gpus", "2"]
    gpus = int(args[args.index("--gpus") + 1]) if "--gpus" in args else 1
    out = os.path.join(ROOT, "gpurun_out", "race_trace")
    os.makedirs(out, exist_ok=True)
    env = {"SCALING_AMD_SINGLE_STREAM": os.environ.get("SCALING_AMD_SINGLE_STREAM", "1"),
           "SCALING_AMD_DETERMINISTIC": "1",
           "SCALING_AMD_BENCH_TRACE_GRADS": os.environ.get("SCALING_AMD_BENCH_TRACE_GRADS", "1")}
    runs = int(os.environ.get("RACE_TRACE_RUNS", "2"))
    for i in range(runs):
        for r in range(gpus):
            p = os.path.join(out, f"run{i}.rank{r}.jsonl")
            if os.path.exists(p):
                os.remove(p)
        run(args, os.path.join(out, f"run{i}"), env)
    for k in range(1, runs):
        for r in range(gpus):
            a, b = load(os.path.join(out, "run0"), r), load(os.path.join(out, f"run{k}"), r)
            first = None
            for x, y in zip(a, b):
                for key in ("loss", "gtrace", "pgrads_pre", "pgrads", "grads", "grad_norm", "params"):
                    if key not in x:
                        continue
                    if key == "gtrace" and x[key] != y[key]:
                        idx = [j for j, (u, v) in enumerate(zip(x[key], y[key])) if u != v]
                        j0 = idx[0]
                        names = [x[key][j][0] for j in idx[:12]]
                        print(f"   step {x['step']}: {len(idx)} of {len(x[key])} trace entries differ, first: {names}",
                              flush=True)
                        first = (x["step"], f"gtrace: first differing input gradient #{j0} of {len(x[key])} "
                                 f"(backward order) entering {x[key][j0][0]}: {x[key][j0][1]} vs {y[key][j0][1]}; "
                                 f"previous entries: {[e[0] for e in x[key][max(0, j0 - 3):j0]]}",
                                 x["loss"], y["loss"])
                        break
                    if x[key] != y[key]:
                        diff = key
                        if isinstance(x[key], list):
                            idx = [j for j, (u, v) in enumerate(zip(x[key], y[key])) if u != v]
                            diff = f"{key} (indices {idx[:8]}{'...' if len(idx) > 8 else ''} of {len(x[key])})"
                            if key in ("pgrads_pre", "pgrads", "params"):
                                names = a[0].get("names") or []
                                diff += " " + str([names[j] for j in idx[:8]] if names else "")
                        first = (x["step"], diff, x["loss"], y["loss"])
                        break
                if first:
                    break
            print(f"run {k} vs run 0, rank {r}: " + ("identical" if first is None else
                  f"first difference at step {first[0]}: {first[1]} (loss {first[2]} vs {first[3]})"), flush=True)


if __name__ == "__main__":
    main()
