// TEMPORARY probe: where the NT GEMM's cycles go.  Built once per NT_PROBE value (see gemm_nt.hip), each binary
// times the kernel at the 7B shapes; 0 is the real kernel, the others remove one constraint (results are garbage).
#include "../csrc/kernels/gemm_nt.hip"
#include <cstdio>

__global__ void fill(uint16_t* p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 15;
        p[i] = (uint16_t)(0x3c00 + (h & 0x1ff));  // bf16 in [2^-7, 2^-6)
    }
}

int main() {
    const int M = 32768;
    struct S { const char* n; int N, K; } sh[] = {
        {"qkv", 6144, 4096}, {"mlp_in", 22016, 4096}, {"mlp_out", 4096, 11008}, {"dgrad_mlp_in", 4096, 22016}};
    const size_t na = (size_t)M * 22016, nb = (size_t)22016 * 4096, nc = (size_t)M * 22016;
    uint16_t *A, *B, *C;
    if (hipMalloc(&A, na * 2) || hipMalloc(&B, nb * 2) || hipMalloc(&C, nc * 2)) return 1;
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, A, na, 1u);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, B, nb, 2u);
    hipFuncSetAttribute((const void*)sa_gemm_nt::gemm_nt_kernel<EPI_STORE>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, sa_gemm_nt::kLds);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (auto& s : sh) {
        if (!sa_launch::gemm_nt_supported(M, s.N, s.K, s.K, s.K)) return 2;
        NtEpi ep{};
        ep.C = C;
        ep.ldc = s.N;
        for (int w = 0; w < 3; ++w) sa_launch::gemm_nt(EPI_STORE, A, s.K, B, s.K, M, s.N, s.K, ep, 0);
        float best = 1e30f;
        for (int r = 0; r < 3; ++r) {
            hipEventRecord(e0, 0);
            for (int i = 0; i < 10; ++i) sa_launch::gemm_nt(EPI_STORE, A, s.K, B, s.K, M, s.N, s.K, ep, 0);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms / 10 < best ? ms / 10 : best;
        }
        printf("probe %d %-14s %.3f ms  %.1f TF/s\n", NT_PROBE, s.n, best, 2.0 * M * s.N * s.K / best / 1e9);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    return 0;
}
