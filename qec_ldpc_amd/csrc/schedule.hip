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
// index).  The order inside one (chunk, bucket) depends on LDS-atomic timing and is not
// deterministic, which is harmless for the same reason.
//
// Counting sort over kBuckets weight buckets (integer/byte work, HBM/L2-bound) in three
// launches with no global atomics (same-address atomics from every workgroup serialise at L2):
//   hist    : one workgroup per chunk of consecutive syndromes, four threads per syndrome
//             (16-byte loads along a quarter of its rows, 8 in flight); the workgroup
//             histograms the buckets in LDS and stores its counts [chunk][bucket]
//   offsets : one workgroup; four threads per bucket sum a quarter of the chunks each, the
//             bucket totals are scanned heaviest-first, and every (chunk, bucket) count is
//             replaced by that chunk's first position in the bucket
//   scatter : each chunk's workgroup places its syndromes from its own offsets (LDS atomics),
//             perm[pos] = b
#include <hip/hip_runtime.h>

#include <cstdint>

#include "qec_internal.h"

namespace qec {

constexpr int kBuckets = 256;    // bucket k = 255 - min(weight, 255): 0 = heaviest
constexpr int kSchedThreads = 256;
constexpr int kHistThreads = 1024;
constexpr int kHistSplit = 4;    // threads per syndrome in the weight pass
constexpr int kOffThreads = 1024;
constexpr int kOffSplit = kOffThreads / kBuckets;  // threads per bucket in the offsets pass
constexpr int kMaxChunks = 1024;
constexpr int kMinChunk = 256;   // rows per chunk
constexpr int kMaxChunk = 4096;

// Weight (bit 0 of each byte) of bytes [g0, g1) of s, read by one thread with 16-byte loads at
// aligned addresses; bytes outside the range are masked off (the first and last loads may
// straddle it; they are read whole, which never leaves the pages the batch lies in).
__device__ __forceinline__ uint32_t range_weight(const uint8_t* s, long long lo, long long hi)
{
    const uintptr_t g0 = reinterpret_cast<uintptr_t>(s + lo), g1 = reinterpret_cast<uintptr_t>(s + hi);
    uint32_t sum = 0;
    // 8 loads in flight per round (all issued before the first is used)
    for (uintptr_t a0 = g0 & ~(uintptr_t)15; a0 < g1; a0 += 16 * 8) {
        uint4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            v[j] = a0 + 16 * j < g1 ? *reinterpret_cast<const uint4*>(a0 + 16 * j) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t w[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uintptr_t o = a0 + 16 * j + 4 * k;
                uint32_t x = w[k] & 0x01010101u;
                if (o < g0) x = (g0 - o) >= 4 ? 0u : x & (0xFFFFFFFFu << (8 * (int)(g0 - o)));
                if (o + 4 > g1) x = o >= g1 ? 0u : x & (0xFFFFFFFFu >> (8 * (int)(o + 4 - g1)));
                sum += __popc(x);
            }
        }
    }
    return sum;
}

// ctr[0, 256): bucket totals, ctr[256, 512): bucket cursors (zeroed by the launch)
// kHistSplit adjacent lanes per syndrome, each summing a quarter of its sX row and of its sZ
// row; the quarters are added with lane shuffles
__global__ __launch_bounds__(kHistThreads) void schedule_hist_kernel(const uint8_t* __restrict__ sX,
                                                                   const uint8_t* __restrict__ sZ, long long B,
                                                                   int mX, int mZ, int chunk,
                                                                   uint8_t* __restrict__ key,
                                                                   uint32_t* __restrict__ counts,
                                                                   uint8_t* __restrict__ zero_flags)
{
    __shared__ uint32_t h[kBuckets];
    const int t = threadIdx.x;
    const int q = t % kHistSplit;
    const long long r0 = (long long)blockIdx.x * chunk;
    const long long r1 = r0 + chunk < B ? r0 + chunk : B;
    if (t < kBuckets) h[t] = 0;
    __syncthreads();
    for (long long b = r0 + t / kHistSplit; b - (t / kHistSplit) < r1; b += kHistThreads / kHistSplit) {
        uint32_t w = 0;
        if (b < r1) {
            const long long x0 = b * mX + (long long)(mX * q / kHistSplit), x1 = b * mX + (long long)(mX * (q + 1) / kHistSplit);
            const long long z0 = b * mZ + (long long)(mZ * q / kHistSplit), z1 = b * mZ + (long long)(mZ * (q + 1) / kHistSplit);
            w = range_weight(sX, x0, x1) + range_weight(sZ, z0, z1);
        }
#pragma unroll
        for (int o = 1; o < kHistSplit; o <<= 1) w += __shfl_xor(w, o);
        if (q == 0 && b < r1) {
            const int bk = kBuckets - 1 - (int)(w < kBuckets - 1 ? w : kBuckets - 1);
            key[b] = (uint8_t)bk;
            atomicAdd(&h[bk], 1u);
            if (zero_flags) zero_flags[b] = 0;  // sector-split launches OR their flags in
        }
    }
    __syncthreads();
    if (t < kBuckets) counts[(long long)blockIdx.x * kBuckets + t] = h[t];
}

// counts[c][k] -> position of chunk c's first syndrome of bucket k.  kOffSplit threads per
// bucket, each over a contiguous range of chunks, loaded kOffBatch at a time into registers.
constexpr int kOffBatch = 32;
__global__ __launch_bounds__(kOffThreads) void schedule_offsets_kernel(uint32_t* __restrict__ counts, int nch)
{
    __shared__ uint32_t part[kOffSplit][kBuckets];
    __shared__ uint32_t base[kBuckets];
    const int k = threadIdx.x % kBuckets, q = threadIdx.x / kBuckets;
    const int c0 = nch * q / kOffSplit, c1 = nch * (q + 1) / kOffSplit;
    uint32_t sum = 0;
    for (int cb = c0; cb < c1; cb += kOffBatch) {
        uint32_t v[kOffBatch];
#pragma unroll
        for (int j = 0; j < kOffBatch; ++j) v[j] = cb + j < c1 ? counts[(cb + j) * kBuckets + k] : 0u;
#pragma unroll
        for (int j = 0; j < kOffBatch; ++j) sum += v[j];
    }
    part[q][k] = sum;
    __syncthreads();
    if (q == 0) {
        uint32_t tot = 0;
#pragma unroll
        for (int j = 0; j < kOffSplit; ++j) tot += part[j][k];
        base[k] = tot;
    }
    __syncthreads();
    for (int o = 1; o < kBuckets; o <<= 1) {  // inclusive scan of the bucket totals
        const uint32_t add = (q == 0 && k >= o) ? base[k - o] : 0u;
        __syncthreads();
        if (q == 0) base[k] += add;
        __syncthreads();
    }
    uint32_t run = (k ? base[k - 1] : 0u);  // exclusive
#pragma unroll
    for (int j = 0; j < kOffSplit; ++j)
        if (j < q) run += part[j][k];
    for (int cb = c0; cb < c1; cb += kOffBatch) {
        uint32_t v[kOffBatch];
#pragma unroll
        for (int j = 0; j < kOffBatch; ++j) v[j] = cb + j < c1 ? counts[(cb + j) * kBuckets + k] : 0u;
#pragma unroll
        for (int j = 0; j < kOffBatch; ++j) {
            if (cb + j < c1) counts[(cb + j) * kBuckets + k] = run;
            run += v[j];
        }
    }
}

__global__ __launch_bounds__(kSchedThreads) void schedule_scatter_kernel(const uint8_t* __restrict__ key, long long B,
                                                                       int chunk,
                                                                       const uint32_t* __restrict__ offsets,
                                                                       int32_t* __restrict__ perm)
{
    __shared__ uint32_t cur[kBuckets];
    const int t = threadIdx.x;
    cur[t] = offsets[(long long)blockIdx.x * kBuckets + t];  // kSchedThreads == kBuckets
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

// workspace layout: perm [B] i32, counts [chunks][256] u32, key [B] u8
static size_t perm_bytes(long long B) { return ((size_t)B * sizeof(int32_t) + 255) & ~(size_t)255; }

size_t schedule_workspace_bytes(long long B, int, int)
{
    return perm_bytes(B) + (size_t)kMaxChunks * kBuckets * 4 + B + 64;
}

// Fills the workspace (schedule_workspace_bytes bytes) and returns in *perm_out the
// heaviest-first order of the batch.  zero_flags (nullable): B bytes the hist pass zeroes on
// the way (the sector-split decode ORs its flags into them).
int launch_schedule(const uint8_t* sX, const uint8_t* sZ, long long B, int mX, int mZ, void* ws,
                    uint8_t* zero_flags, int32_t** perm_out, hipStream_t st)
{
    if (B > schedule_max_batch()) return fail(QEC_ERR_ARG, "schedule: batch too large to order");
    int nch = 0;
    const int chunk = chunk_of(B, &nch);
    uint8_t* p = static_cast<uint8_t*>(ws);
    int32_t* perm = reinterpret_cast<int32_t*>(p);
    uint32_t* counts = reinterpret_cast<uint32_t*>(p + perm_bytes(B));
    uint8_t* key = reinterpret_cast<uint8_t*>(counts + (size_t)kMaxChunks * kBuckets);
    *perm_out = perm;
    hipLaunchKernelGGL(schedule_hist_kernel, dim3(nch), dim3(kHistThreads), 0, st, sX, sZ, B, mX, mZ, chunk, key,
                       counts, zero_flags);
    hipLaunchKernelGGL(schedule_offsets_kernel, dim3(1), dim3(kOffThreads), 0, st, counts, nch);
    hipLaunchKernelGGL(schedule_scatter_kernel, dim3(nch), dim3(kSchedThreads), 0, st, key, B, chunk, counts, perm);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) return fail(QEC_ERR_HIP, std::string("schedule launch: ") + hipGetErrorString(err));
    return QEC_OK;
}

}  // namespace qec
