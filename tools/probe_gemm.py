"""Probe: device info + hipBLASLt bf16 GEMM throughput for Llama-7B shapes."""
import torch, time, json, os
print(torch.__version__, torch.version.hip, torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0))
dev = "cuda"
res = {}
def bench(M, N, K, trans_b=True, iters=20):
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        c = torch.nn.functional.linear(a, b)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        c = torch.nn.functional.linear(a, b)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / iters
    return 2 * M * N * K / dt / 1e12
for M in (4096, 8192, 16384):
    for (N, K) in ((12288, 4096), (6144, 4096), (4096, 4096), (22016, 4096), (4096, 11008), (32000, 4096)):
        tf = bench(M, N, K)
        res[f"{M}x{N}x{K}"] = round(tf, 1)
        print(M, N, K, f"{tf:.1f} TF", flush=True)
# backward-shaped GEMMs: dW = dY^T X  (N x M) @ (M x K)
for M in (8192,):
    for (N, K) in ((12288, 4096), (22016, 4096), (4096, 11008)):
        dy = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        for _ in range(3): w = dy.t() @ x
        torch.cuda.synchronize(); t = time.perf_counter()
        for _ in range(20): w = dy.t() @ x
        torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 20
        print("dW", M, N, K, f"{2*M*N*K/dt/1e12:.1f} TF", flush=True)
# SDPA reference (torch's own) for scale
q = torch.randn(2, 32, 4096, 128, device=dev, dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(2, 32, 4096, 128, device=dev, dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(2, 32, 4096, 128, device=dev, dtype=torch.bfloat16, requires_grad=True)
for _ in range(3):
    o = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True)
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(10):
    o = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True)
torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 10
fl = 4 * 2 * 32 * 4096 * 4096 * 128 / 2
print("sdpa fwd causal", f"{fl/dt/1e12:.1f} TF", dt * 1e3, "ms", flush=True)
g = torch.randn_like(o)
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(5):
    o = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True)
    o.backward(g)
torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 5
print("sdpa fwd+bwd causal", f"{3.5*fl/dt/1e12:.1f} TF", dt * 1e3, "ms", flush=True)
print("mem", torch.cuda.get_device_properties(0).total_memory / 2**30, "GiB")
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/probe_gemm.json", "w"))
