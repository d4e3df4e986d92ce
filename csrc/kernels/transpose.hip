// 2-byte (bf16 / fp16) matrix transpose out[C][R] = in[R][C] for the dgrad weight cache: the backward
// GEMM dX = dY W then runs as dY (W^T)^T, the layout hipBLASLt reaches its forward-GEMM rate on.
//  * 64 x 64 tile per 256-thread workgroup; 16-B loads (8 elements per lane, 8 lanes per 128-B row
//    segment) into an LDS image padded to 72 elements per row (odd multiple of 16 B between rows, so the
//    column reads of the store pass spread over the banks), 16-B stores of 8 consecutive output elements.
//  * grid: x over column tiles, y over row tiles; rows/cols multiples of 64 (host checks), row stride
//    ld_in elements (a fused [q; k; v] view is one matrix).
#include "common.h"
#include "launch.h"

using namespace sa;

namespace {
constexpr int kT = 64, kPad = 72;

__global__ __launch_bounds__(256) void transpose_u16_kernel(const u16* __restrict__ in, int64_t ld_in,
                                                            u16* __restrict__ out, int64_t R) {
    __shared__ u16 tile[kT * kPad];
    const int64_t r0 = (int64_t)blockIdx.y * kT, c0 = (int64_t)blockIdx.x * kT;
    const int t = threadIdx.x;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int row = p * 32 + (t >> 3), seg = (t & 7) * 8;
        const u16x8 v = *reinterpret_cast<const u16x8*>(in + (r0 + row) * ld_in + c0 + seg);
        *reinterpret_cast<u16x8*>(&tile[row * kPad + seg]) = v;
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int orow = p * 32 + (t >> 3), seg = (t & 7) * 8;  // output row = input column
        u16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = tile[(seg + j) * kPad + orow];
        *reinterpret_cast<u16x8*>(out + (c0 + orow) * R + r0 + seg) = v;
    }
}
}  // namespace

namespace sa_launch {
bool transpose_supported(int64_t R, int64_t C, int64_t ld_in) {
    return R > 0 && C > 0 && R % kT == 0 && C % kT == 0 && ld_in % 8 == 0 && C / kT < (int64_t(1) << 31) &&
           R / kT < 65536;
}
void transpose_u16(const void* in, int64_t ld_in, void* out, int64_t R, int64_t C, hipStream_t st) {
    hipLaunchKernelGGL(transpose_u16_kernel, dim3((unsigned)(C / kT), (unsigned)(R / kT)), dim3(256), 0, st,
                       (const u16*)in, ld_in, (u16*)out, R);
}
}  // namespace sa_launch
