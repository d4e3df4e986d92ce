"""Bisects a multi- vs single-stream difference of the race check (tests/test_gpu_rehearsal.py): runs one bench layout
with every side stream on (multi), every side stream folded (single), and each feature of
scaling_amd.core.utils.debug_env.SIDE_STREAM_FEATURES folded alone, and prints (param checksum, loss) per mode.

    python tools/race_bisect.py [bench args ...]     (default: --gpus 2, the DP2 case)
    python tools/race_bisect.py --repeat [bench args ...]   run-to-run determinism (single stream) per GEMM setting
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASE = ["--model", "llama_tiny", "--backend", "gloo-gpu", "--seq-len", "256", "--micro-batch", "2", "--steps", "3",
        "--warmup", "1"]


def run(args, env_extra):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.update(env_extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *BASE, *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        return ("FAILED", r.stderr[-2000:])
    res = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][0]["config"]
    return (res["param_checksum"], res["loss"])


def main():
    rep = "--repeat" in sys.argv
    args = [a for a in sys.argv[1:] if a != "--repeat"] or ["--gpus", "2"]
    if rep:  # run-to-run determinism per GEMM backend, streams folded and not
        modes = []
        variants = (("default", {}),
                    ("rocblas-noatomics", {"SCALING_AMD_GEMM_TUNING": "off", "TORCH_BLAS_PREFER_HIPBLASLT": "0",
                                           "ROCBLAS_DEFAULT_ATOMICS_MODE": "0"}),
                    ("torch-deterministic", {"SCALING_AMD_DETERMINISTIC": "1"}),
                    ("rocblas-deterministic", {"SCALING_AMD_DETERMINISTIC": "1", "SCALING_AMD_GEMM_TUNING": "off",
                                               "TORCH_BLAS_PREFER_HIPBLASLT": "0"}))
        for tag, env in variants:
            for i in range(2):
                modes.append((f"single/{tag}#{i}", {**env, "SCALING_AMD_SINGLE_STREAM": "1"}))
        out = {}
        for name, env in modes:
            out[name] = run(args, env)
            print(f"{' '.join(args)} | {name:22s} | {out[name]}", flush=True)
        return
    det = {"SCALING_AMD_DETERMINISTIC": "1"}  # as the race-check test: vendor kernels deterministic
    modes = [("multi", dict(det)), ("single", {**det, "SCALING_AMD_SINGLE_STREAM": "1"})]
    for f in ("dp_comm", "opt_step", "wgrad", "tp_comm"):
        modes.append((f"fold:{f}", {**det, "SCALING_AMD_SINGLE_STREAM": f}))
    modes.append(("multi-again", dict(det)))
    out = {}
    for name, env in modes:
        out[name] = run(args, env)
        same = out[name] == out.get("single")
        print(f"{' '.join(args)} | {name:14s} | equals single: {same} | {out[name]}", flush=True)


if __name__ == "__main__":
    main()
