// Dispatch order of a decode launch (QEC_OPT_SCHEDULE): heaviest syndromes first.
//
// A fixed-iteration launch ends when its slowest wave ends.  Almost every P61 sector
// reaches a hard (all 0/1) 2-cycle within a handful of iterations and then jumps to the
// end (bp_decode.hip, cycle_end), but a few per 10^4 never do and run every iteration
// in full arithmetic -- about 10x an average wave.  Dispatched in batch order, such a
// wave can start near the end of the launch and extend it (measured: 11 such sectors
// in 65 536 P61 syndromes at p = 0.01 cost 15 % of the launch).  Syndrome weight
// predicts them (more unsatisfied checks, more errors), so the waves take syndromes
// in descending weight: the long ones start first and their tail hides behind the
// bulk, and waves of one workgroup / CU see similar work.
//
// Only the order in which waves pick syndromes changes; every syndrome's arithmetic,
// and so every output bit, is the same (outputs are written at the syndrome's own
// index).  The order inside one weight bucket depends on atomic timing and is not
// deterministic, which is harmless for the same reason.
//
// Counting sort over kBuckets weight buckets (integer/byte work, HBM/L2-bound): a memset of
// the 2 x 256 bucket counters and two launches:
//   hist    : one workgroup per chunk of consecutive syndromes, four threads per syndrome
//             (16-byte loads along a quarter of its rows); the workgroup histograms the buckets in LDS,
//             stores its counts and adds them to the bucket totals (one global atomic per
//             non-empty bucket)
//   scatter : each chunk's workgroup scans the bucket totals (heaviest first) in LDS,
//             reserves its range in every bucket with one atomic, and places its syndromes
//             there (LDS atomics), perm[pos] = b
#include <hip/hip_runtime.h>

#include <cstdint>

#include "qec_internal.h"

namespace qec {

constexpr int kBuckets = 256;    // bucket k = 255 - min(weight, 255): 0 = heaviest
constexpr int kSchedThreads = 256;
constexpr int kMaxChunks = 1024;
constexpr int kHistThreads = 1024;
constexpr int kHistSplit = 4;    // threads per syndrome in the weight pass
constexpr int kMinChunk = 256;   // rows per chunk
constexpr int kMaxChunk = 4096;

// Weight (bit 0 of each byte) of bytes [g0, g1) of s, read by one thread with 16-byte loads at
// aligned addresses; bytes outside the range are masked off (the first and last loads may
// straddle it; they are read whole, which never leaves the pages the batch lies in).
__device__ __forceinline__ uint32_t range_weight(const uint8_t* s, long long lo, long long hi)
{
    const uintptr_t g0 = reinterpret_cast<uintptr_t>(s + lo), g1 = reinterpret_cast<uintptr_t>(s + hi);
    uint32_t sum = 0;
    for (uintptr_t a = g0 & ~(uintptr_t)15; a < g1; a += 16) {
        const uint4 v = *reinterpret_cast<const uint4*>(a);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uintptr_t o = a + 4 * k;
            uint32_t x = w[k] & 0x01010101u;
            if (o < g0) x = (g0 - o) >= 4 ? 0u : x & (0xFFFFFFFFu << (8 * (int)(g0 - o)));
            if (o + 4 > g1) x = o >= g1 ? 0u : x & (0xFFFFFFFFu >> (8 * (int)(o + 4 - g1)));
            sum += __popc(x);
        }
    }
    return sum;
}

// ctr[0, 256): bucket totals, ctr[256, 512): bucket cursors (zeroed by the launch)
// kHistSplit threads per syndrome, each summing a quarter of its sX row and of its sZ row
__global__ __launch_bounds__(kHistThreads) void schedule_hist_kernel(const uint8_t* __restrict__ sX,
                                                                   const uint8_t* __restrict__ sZ, long long B,
                                                                   int mX, int mZ, int chunk,
                                                                   uint8_t* __restrict__ key,
                                                                   uint32_t* __restrict__ counts,
                                                                   uint32_t* __restrict__ ctr)
{
    __shared__ uint32_t h[kBuckets];
    __shared__ uint32_t wt[kHistThreads / kHistSplit];
    const int t = threadIdx.x;
    const int q = t % kHistSplit, rl = t / kHistSplit;  // quarter, row within the pass
    constexpr int kRows = kHistThreads / kHistSplit;
    const long long r0 = (long long)blockIdx.x * chunk;
    const long long r1 = r0 + chunk < B ? r0 + chunk : B;
    if (t < kBuckets) h[t] = 0;
    for (long long p0 = r0; p0 < r1; p0 += kRows) {
        if (t < kRows) wt[t] = 0;
        __syncthreads();
        const long long b = p0 + rl;
        if (b < r1) {
            const long long x0 = b * mX + (long long)mX * q / kHistSplit, x1 = b * mX + (long long)mX * (q + 1) / kHistSplit;
            const long long z0 = b * mZ + (long long)mZ * q / kHistSplit, z1 = b * mZ + (long long)mZ * (q + 1) / kHistSplit;
            const uint32_t w = range_weight(sX, x0, x1) + range_weight(sZ, z0, z1);
            if (w) atomicAdd(&wt[rl], w);
        }
        __syncthreads();
        if (t < kRows && p0 + t < r1) {
            const uint32_t w = wt[t];
            const int bk = kBuckets - 1 - (int)(w < kBuckets - 1 ? w : kBuckets - 1);
            key[p0 + t] = (uint8_t)bk;
            atomicAdd(&h[bk], 1u);
        }
        __syncthreads();
    }
    if (t < kBuckets) {
        const uint32_t c = h[t];
        counts[(long long)blockIdx.x * kBuckets + t] = c;
        if (c) atomicAdd(&ctr[t], c);
    }
}

__global__ __launch_bounds__(kSchedThreads) void schedule_scatter_kernel(const uint8_t* __restrict__ key, long long B,
                                                                       int chunk,
                                                                       const uint32_t* __restrict__ counts,
                                                                       uint32_t* __restrict__ ctr,
                                                                       int32_t* __restrict__ perm)
{
    __shared__ uint32_t cur[kBuckets];
    const int t = threadIdx.x;
    uint32_t tot = 0;
    if (t < kBuckets) cur[t] = tot = ctr[t];
    __syncthreads();
    for (int o = 1; o < kBuckets; o <<= 1) {  // inclusive scan of the totals, heaviest bucket first
        const uint32_t add = (t < kBuckets && t >= o) ? cur[t - o] : 0u;
        __syncthreads();
        if (t < kBuckets) cur[t] += add;
        __syncthreads();
    }
    if (t < kBuckets) {
        const uint32_t c = counts[(long long)blockIdx.x * kBuckets + t];
        cur[t] = cur[t] - tot + (c ? atomicAdd(&ctr[kBuckets + t], c) : 0u);
    }
    __syncthreads();
    const long long r0 = (long long)blockIdx.x * chunk;
    const long long r1 = r0 + chunk < B ? r0 + chunk : B;
    for (long long b = r0 + t; b < r1; b += kSchedThreads) perm[atomicAdd(&cur[key[b]], 1u)] = (int32_t)b;
}

// rows per chunk: at least kMinChunk, enough that there are at most kMaxChunks chunks
static int chunk_of(long long B, int* nchunks)
{
    long long chunk = (B + kMaxChunks - 1) / kMaxChunks;
    if (chunk < kMinChunk) chunk = kMinChunk;
    *nchunks = (int)((B + chunk - 1) / chunk);
    return (int)chunk;
}

// B <= kMaxChunks * kMaxChunk syndromes per ordered launch (4 M)
long long schedule_max_batch() { return (long long)kMaxChunks * kMaxChunk; }

static size_t perm_bytes(long long B) { return ((size_t)B * sizeof(int32_t) + 255) & ~(size_t)255; }

size_t schedule_workspace_bytes(long long B, int, int)
{
    return perm_bytes(B) + (size_t)(kMaxChunks + 2) * kBuckets * 4 + B + 64;
}

// Fills the workspace (schedule_workspace_bytes bytes) and returns in *perm_out the
// heaviest-first order of the batch.
int launch_schedule(const uint8_t* sX, const uint8_t* sZ, long long B, int mX, int mZ, void* ws, int32_t** perm_out,
                    hipStream_t st)
{
    if (B > schedule_max_batch()) return fail(QEC_ERR_ARG, "schedule: batch too large to order");
    int nch = 0;
    const int chunk = chunk_of(B, &nch);
    uint8_t* p = static_cast<uint8_t*>(ws);
    int32_t* perm = reinterpret_cast<int32_t*>(p);
    uint32_t* ctr = reinterpret_cast<uint32_t*>(p + perm_bytes(B));
    uint32_t* counts = ctr + 2 * kBuckets;
    uint8_t* key = reinterpret_cast<uint8_t*>(counts + (size_t)kMaxChunks * kBuckets);
    *perm_out = perm;
    if (hipMemsetAsync(ctr, 0, 2 * kBuckets * sizeof(uint32_t), st) != hipSuccess)
        return fail(QEC_ERR_HIP, "schedule: hipMemsetAsync failed");
    hipLaunchKernelGGL(schedule_hist_kernel, dim3(nch), dim3(kHistThreads), 0, st, sX, sZ, B, mX, mZ, chunk, key,
                       counts, ctr);
    hipLaunchKernelGGL(schedule_scatter_kernel, dim3(nch), dim3(kSchedThreads), 0, st, key, B, chunk, counts, ctr,
                       perm);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) return fail(QEC_ERR_HIP, std::string("schedule launch: ") + hipGetErrorString(err));
    return QEC_OK;
}

}  // namespace qec
