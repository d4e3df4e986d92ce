// Floor of an atomic-dQ ("non-deterministic") flash-attention backward on MI355X at the 7B bench shape.
//
// A one-pass backward (dK/dV workgroup also computes its dQ contribution) must add, per (key block, 32-row
// query tile) pair that the causal mask leaves, a 32 x D fp32 tile into the global dQ accumulator.  This
// program issues exactly that atomic traffic -- no-return global_atomic_add_f32, one register of a 32x32
// accumulator per wave-instruction (two 128-B row segments: the full-rate shape) -- for one layer
// (8 sequences x 4096 tokens, 32 q heads, D 128, 256-key blocks) and times it.  x 32 layers = the per-step
// floor that such a kernel cannot beat, to compare with the deterministic two-kernel backward's dQ pass.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/atomic_dq_floor tools/atomic_dq_floor.hip && tools/atomic_dq_floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int S = 4096, H = 32, B = 8, D = 128, KB = 256, QT = 32;

// one workgroup (4 waves) per (seq, head, key block); waves split the block's causal query tiles
__global__ __launch_bounds__(256) void dq_atomic_kernel(float* __restrict__ dq, float v) {
    const int kb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q_first = kb * KB / QT;  // causal: query tiles at or after the key block
    float* base = dq + ((size_t)b * H + h) * (size_t)S * D;
    for (int qt = q_first + wave; qt < S / QT; qt += 4) {
        // 32 x 128 tile = 4 accumulators of 32 x 32; register r of an accumulator: rows 8(r/4)+r%4 (+4 for the
        // upper 32 lanes), column lane & 31
#pragma unroll
        for (int t = 0; t < D / 32; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = qt * QT + 8 * (r >> 2) + (r & 3) + 4 * (lane >> 5);
                float* p = base + (size_t)row * D + 32 * t + (lane & 31);
                __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
    }
}

int main() {
    const size_t n = (size_t)B * H * S * D;
    float* dq = nullptr;
    if (hipMalloc(&dq, n * sizeof(float)) != hipSuccess) return 1;
    (void)hipMemset(dq, 0, n * sizeof(float));
    dim3 grid(S / KB, H, B);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(dq_atomic_kernel, grid, 256, 0, 0, dq, 1.0f);  // warm-up
    (void)hipDeviceSynchronize();
    std::vector<float> ms;
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(dq_atomic_kernel, grid, 256, 0, 0, dq, 1.0f);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float t = 0.f;
        (void)hipEventElapsedTime(&t, e0, e1);
        ms.push_back(t);
    }
    double tiles = 0;
    for (int kb = 0; kb < S / KB; ++kb) tiles += S / QT - kb * KB / QT;
    const double bytes = tiles * H * B * QT * D * 4.0;
    float best = ms[0];
    for (float t : ms) best = t < best ? t : best;
    // check: element (row, d) received one add per key block at or before its row's block
    std::vector<float> h(D * 2);
    (void)hipMemcpy(h.data(), dq + (size_t)(S - 1) * D, D * sizeof(float), hipMemcpyDeviceToHost);
    printf("{\"atomic_bytes_per_layer_GB\": %.3f, \"ms_per_layer_best\": %.3f, \"TB_per_s\": %.3f, "
           "\"ms_per_step_32_layers\": %.1f, \"last_row_adds\": %.0f, \"expected_adds\": %d}\n",
           bytes / 1e9, best, bytes / (best * 1e-3) / 1e12, best * 32.0, h[0], 6 * (S / KB));
    (void)hipFree(dq);
    return 0;
}
