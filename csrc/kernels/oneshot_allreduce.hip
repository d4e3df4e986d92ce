// One-shot all-reduce over IPC-mapped peer buffers for small tensor-parallel messages on one node.
//
// RCCL's ring/tree all-reduce over xGMI costs several link latencies per call; a TP2..TP8 activation-gradient
// all-reduce of a few MiB is latency-bound.  Here every rank of the group owns one registered buffer
// (hipMalloc'd, IPC handle exchanged once) holding two data slots (even / odd call) and a flag row; a call:
//   1. the caller copies its input into its own slot (stream-ordered D2D copy, before this kernel);
//   2. block 0 publishes it: system-scope release, then epoch -> flag[my rank] in every PEER's flag row
//      (vector stores over xGMI);
//   3. every block waits until its own flag row holds `epoch` from all ranks (bounded spin: on timeout it
//      records an error word, skips the sum and fills its part of the output with NaN, so a missing peer can
//      neither hang the GPU nor turn stale slots into plausible numbers), system-scope acquire;
//   4. each thread sums its 16-B chunks from all ranks' slots in fp32 and writes the result.
// The error word is read back at the optimizer's per-step host sync (custom_allreduce.pending_error_words),
// which raises: a timeout is never silent.
// Double-buffered slots make one barrier per call sufficient: a peer that reached call e's barrier has
// finished reading call e-1, whose slot call e+1 reuses.  All flag traffic uses vector memory instructions.
#include <algorithm>

#include "common.h"
#include "launch.h"

using namespace sa;

namespace {

template <typename T> struct Vec;
template <> struct Vec<u16> {  // bf16
    static constexpr int N = 8;
    __device__ static void add(const void* p, float* acc) {
        const u16x8 v = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
    }
    __device__ static void st(void* p, const float* acc) {
        u16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = f2bf(acc[j]);
        *reinterpret_cast<u16x8*>(p) = v;
    }
};
template <> struct Vec<_Float16> {
    static constexpr int N = 8;
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    __device__ static void add(const void* p, float* acc) {
        const h8 v = *reinterpret_cast<const h8*>(p);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += (float)v[j];
    }
    __device__ static void st(void* p, const float* acc) {
        h8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (_Float16)acc[j];
        *reinterpret_cast<h8*>(p) = v;
    }
};
template <> struct Vec<float> {
    static constexpr int N = 4;
    __device__ static void add(const void* p, float* acc) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(p);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += v[j];
    }
    __device__ static void st(void* p, const float* acc) {
        *reinterpret_cast<f32x4*>(p) = f32x4{acc[0], acc[1], acc[2], acc[3]};
    }
};

constexpr int kMaxRanks = 8;
struct Peers {
    char* base[kMaxRanks];  // registered buffer of every rank (own one included), mapped in this process
};

// T elements; n a multiple of the vector width (host checks); out may alias nothing in the buffers
template <typename T>
__global__ __launch_bounds__(256) void oneshot_allreduce_kernel(Peers peers, int world, int rank, int64_t slot_off,
                                                                int64_t flag_off, uint32_t epoch, int signal,
                                                                void* __restrict__ out, int64_t n, int* err,
                                                                int64_t max_spins) {
    __shared__ int timed_out;
    if (threadIdx.x == 0) timed_out = 0;
    if (signal) {
        if (blockIdx.x == 0 && threadIdx.x < world) {
            __atomic_thread_fence(__ATOMIC_RELEASE);  // the slot copy happened earlier on this stream
            __threadfence_system();
            uint32_t* f = reinterpret_cast<uint32_t*>(peers.base[threadIdx.x] + flag_off) + rank;
            __hip_atomic_store(f, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (threadIdx.x == 0) {
            const uint32_t* mine = reinterpret_cast<const uint32_t*>(peers.base[rank] + flag_off);
            for (int q = 0; q < world; ++q) {
                int64_t spins = 0;
                while (__hip_atomic_load(mine + q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
                    __builtin_amdgcn_s_sleep(2);
                    if (++spins > max_spins) {  // (default ~seconds) a peer never arrived
                        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        timed_out = 1;
                        break;
                    }
                }
                if (timed_out) break;
            }
            __threadfence_system();
        }
    }
    __syncthreads();
    constexpr int V = Vec<T>::N;
    const int64_t nvec = n / V;
    if (timed_out) {  // the peers' slots may hold an earlier call's data: poison instead of summing it
        float nan[V];
#pragma unroll
        for (int j = 0; j < V; ++j) nan[j] = __builtin_nanf("");
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * blockDim.x)
            Vec<T>::st(reinterpret_cast<char*>(out) + i * V * (int64_t)sizeof(T), nan);
        return;
    }
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * blockDim.x) {
        float acc[V];
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] = 0.f;
        for (int q = 0; q < world; ++q) {  // fixed rank order: every rank computes the bit-identical sum
            const char* src = peers.base[q] + slot_off + i * V * (int64_t)sizeof(T);
            Vec<T>::add(src, acc);
        }
        Vec<T>::st(reinterpret_cast<char*>(out) + i * V * (int64_t)sizeof(T), acc);
    }
}

}  // namespace

namespace sa_launch {
void oneshot_allreduce(int dtype, char* const* bases, int world, int rank, int64_t slot_off, int64_t flag_off,
                       uint32_t epoch, bool signal, void* out, int64_t n, int* err, int64_t max_spins,
                       hipStream_t st) {
    Peers p{};
    for (int i = 0; i < world && i < kMaxRanks; ++i) p.base[i] = bases[i];
    const int vec = dtype == DT_F32 ? 4 : 8;
    const int64_t nvec = n / vec;
    const int grid = (int)std::min<int64_t>(std::max<int64_t>((nvec + 255) / 256, 1), 1024);
    if (dtype == DT_BF16)
        hipLaunchKernelGGL(oneshot_allreduce_kernel<u16>, grid, 256, 0, st, p, world, rank, slot_off, flag_off, epoch,
                           signal ? 1 : 0, out, n, err, max_spins);
    else if (dtype == DT_F16)
        hipLaunchKernelGGL(oneshot_allreduce_kernel<_Float16>, grid, 256, 0, st, p, world, rank, slot_off, flag_off, epoch,
                           signal ? 1 : 0, out, n, err, max_spins);
    else
        hipLaunchKernelGGL(oneshot_allreduce_kernel<float>, grid, 256, 0, st, p, world, rank, slot_off, flag_off, epoch,
                           signal ? 1 : 0, out, n, err, max_spins);
}
}  // namespace sa_launch
