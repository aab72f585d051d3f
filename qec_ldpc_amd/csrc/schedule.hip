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
//   offsets : one workgroup per bucket scans its column of the count matrix over the chunks
//             (each chunk's exclusive prefix, in place) and stores the bucket total;
//   scatter : each chunk's workgroup scans the 256 totals heaviest-first, adds its own
//             prefixes, and places its syndromes (LDS atomics), perm[pos] = b.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>

#include "qec_internal.h"

namespace qec {

constexpr int kBuckets = 256;    // bucket k = 255 - min(weight, 255): 0 = heaviest
constexpr int kHistThreads = 1024;
// threads per syndrome in the weight pass: 4 for long rows (P61: 549 bytes), 1 for short ones
// (P7: 42 bytes), where four threads would only multiply the waves of a latency-bound launch
// (8, one round of loads per thread for P61, is slower: 23.8 vs 17.1 us,
// profiles/r01/session7/rocprof_hist_split_s7bb.csv)
constexpr int kHistSplitLong = 4;
constexpr int kShortRows = 128;  // mX + mZ up to this many bytes: one thread per syndrome
constexpr int kMaxChunks = 1024;
constexpr int kMaxChunk = 4096;
// sector-split launches: each sector's waves in the order of that sector's weight
constexpr bool kSchedSectors = true;
constexpr int kTargetChunks = 128;  // chunks (histogram workgroups) aimed for when the batch is small

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

// SPLIT adjacent lanes per syndrome, each summing a 1/SPLIT share of its sX row and of its sZ
// row; the shares are added with lane shuffles
template <int SPLIT>
__device__ __forceinline__ void hist_body(const uint8_t* __restrict__ sX, const uint8_t* __restrict__ sZ, long long B,
                                          int mX, int mZ, int chunk, int nbk, uint8_t* __restrict__ key,
                                          uint32_t* __restrict__ counts, uint32_t* __restrict__ zero_merge,
                                          uint32_t* h)
{
    const int t = threadIdx.x;
    const int q = t % SPLIT;
    const long long r0 = (long long)blockIdx.x * chunk;
    const long long r1 = r0 + chunk < B ? r0 + chunk : B;
    if (t < kBuckets) h[t] = 0;
    __syncthreads();
    for (long long b = r0 + t / SPLIT; b - (t / SPLIT) < r1; b += blockDim.x / SPLIT) {
        uint32_t w = 0;
        if (b < r1) {
            const long long x0 = b * mX + (long long)(mX * q / SPLIT), x1 = b * mX + (long long)(mX * (q + 1) / SPLIT);
            const long long z0 = b * mZ + (long long)(mZ * q / SPLIT), z1 = b * mZ + (long long)(mZ * (q + 1) / SPLIT);
            w = range_weight(sX, x0, x1) + range_weight(sZ, z0, z1);
        }
#pragma unroll
        for (int o = 1; o < SPLIT; o <<= 1) w += __shfl_xor(w, o);
        if (q == 0 && b < r1) {
            const int bk = nbk - 1 - (int)(w < (uint32_t)nbk - 1 ? w : (uint32_t)nbk - 1);
            key[b] = (uint8_t)bk;
            atomicAdd(&h[bk], 1u);
            if (zero_merge) zero_merge[b] = 0u;  // sector-split launches merge their flags there
        }
    }
    __syncthreads();
    if (t < nbk) counts[(long long)blockIdx.x * nbk + t] = h[t];
}

template <int SPLIT>
__global__ __launch_bounds__(kHistThreads) void schedule_hist_kernel(const uint8_t* __restrict__ sX,
                                                                   const uint8_t* __restrict__ sZ, long long B,
                                                                   int mX, int mZ, int chunk, int nbk,
                                                                   uint8_t* __restrict__ key,
                                                                   uint32_t* __restrict__ counts,
                                                                   uint32_t* __restrict__ zero_merge)
{
    __shared__ uint32_t h[kBuckets];
    hist_body<SPLIT>(sX, sZ, B, mX, mZ, chunk, nbk, key, counts, zero_merge, h);
}

// The same weights from bit rows (sX [B][wX], sZ [B][wZ] words; the Monte-Carlo pipeline's
// layout): one thread per syndrome, popcounts of its words.
__device__ __forceinline__ void hist_bits_body(const uint32_t* __restrict__ sX, const uint32_t* __restrict__ sZ,
                                               long long B, int wX, int wZ, int chunk, int nbk,
                                               uint8_t* __restrict__ key, uint32_t* __restrict__ counts,
                                               uint32_t* __restrict__ zero_merge, uint32_t* h)
{
    const int t = threadIdx.x;
    const long long r0 = (long long)blockIdx.x * chunk;
    const long long r1 = r0 + chunk < B ? r0 + chunk : B;
    if (t < kBuckets) h[t] = 0;
    __syncthreads();
    for (long long b = r0 + t; b < r1; b += blockDim.x) {
        uint32_t w = 0;
        for (int k = 0; k < wX; ++k) w += __popc(sX[b * wX + k]);
        for (int k = 0; k < wZ; ++k) w += __popc(sZ[b * wZ + k]);
        const int bk = nbk - 1 - (int)(w < (uint32_t)nbk - 1 ? w : (uint32_t)nbk - 1);
        key[b] = (uint8_t)bk;
        atomicAdd(&h[bk], 1u);
        if (zero_merge) zero_merge[b] = 0u;
    }
    __syncthreads();
    if (t < nbk) counts[(long long)blockIdx.x * nbk + t] = h[t];
}

__global__ __launch_bounds__(kHistThreads) void schedule_hist_bits_kernel(const uint32_t* __restrict__ sX,
                                                                        const uint32_t* __restrict__ sZ, long long B,
                                                                        int wX, int wZ, int chunk, int nbk,
                                                                        uint8_t* __restrict__ key,
                                                                        uint32_t* __restrict__ counts,
                                                                        uint32_t* __restrict__ zero_merge)
{
    __shared__ uint32_t h[kBuckets];
    hist_bits_body(sX, sZ, B, wX, wZ, chunk, nbk, key, counts, zero_merge, h);
}

// Bucket offsets: workgroup k scans column k of the [chunks][256] count matrix (one thread per
// chunk, LDS scan), writes each chunk's exclusive prefix in place and the bucket total.  About
// 2 KiB of the matrix per workgroup; the previous design, every scatter workgroup re-reading
// the whole matrix, moved 1 GiB through L2 at 2^20 syndromes (1024 chunks): 75 us.
constexpr int kScanThreads = 1024;  // = kMaxChunks
__global__ __launch_bounds__(kScanThreads) void schedule_offsets_kernel(int nch, uint32_t* __restrict__ counts,
                                                                        uint32_t* __restrict__ totals)
{
    __shared__ uint32_t v[kScanThreads];
    const int k = blockIdx.x, c = threadIdx.x;
    const uint32_t x = c < nch ? counts[(long long)c * kBuckets + k] : 0u;
    v[c] = x;
    __syncthreads();
    for (int o = 1; o < kScanThreads; o <<= 1) {  // inclusive scan over chunks
        const uint32_t add = c >= o ? v[c - o] : 0u;
        __syncthreads();
        v[c] += add;
        __syncthreads();
    }
    if (c < nch) counts[(long long)c * kBuckets + k] = v[c] - x;  // exclusive: syndromes of bucket k in chunks < c
    if (c == kScanThreads - 1) totals[k] = v[c];
}

// Scatter: workgroup c scans the 256 bucket totals heaviest-first (its bucket starts), adds its
// own chunk prefixes, and places its syndromes (LDS atomics), perm[pos] = b.
constexpr int kScatThreads = 1024;
__global__ __launch_bounds__(kScatThreads) void schedule_scatter_kernel(const uint8_t* __restrict__ key, long long B,
                                                                      int chunk, const uint32_t* __restrict__ prefix,
                                                                      const uint32_t* __restrict__ totals,
                                                                      int32_t* __restrict__ perm)
{
    __shared__ uint32_t start[kBuckets];
    __shared__ uint32_t cur[kBuckets];
    const int t = threadIdx.x;
    const int c = blockIdx.x;
    if (t < kBuckets) start[t] = totals[t];
    __syncthreads();
    for (int o = 1; o < kBuckets; o <<= 1) {  // inclusive scan of the bucket totals, heaviest first
        const uint32_t add = (t < kBuckets && t >= o) ? start[t - o] : 0u;
        __syncthreads();
        if (t < kBuckets) start[t] += add;
        __syncthreads();
    }
    if (t < kBuckets) cur[t] = (t ? start[t - 1] : 0u) + prefix[(long long)c * kBuckets + t];
    __syncthreads();
    const long long r0 = (long long)c * chunk;
    const long long r1 = r0 + chunk < B ? r0 + chunk : B;
    for (long long b = r0 + t; b < r1; b += kScatThreads) perm[atomicAdd(&cur[key[b]], 1u)] = (int32_t)b;
}

// Offsets and scatter in one launch, for at most kMaxFusedChunks chunks: workgroup c reads the whole
// [chunks][256] count matrix (at most 128 KiB, L2-resident after the histogram wrote it), forms the
// bucket totals and its own chunk prefixes in LDS, and scatters as schedule_scatter_kernel.  One
// dependent launch fewer for the batches where the order pass is mostly launch latency (P7 65 536:
// three passes 46 us, of which the 16-workgroup histogram 36 us, profiles/r03/).  It also sizes the
// buckets to the largest possible weight (P7: mX + mZ + 1 = 43 instead of 256: the count matrix
// each workgroup reads shrinks with them).
constexpr int kMaxFusedChunks = 256;
struct FusedLds {
    uint32_t tot[kScatThreads], pre[kScatThreads];  // [part][bucket], part * nbk + k = t
    uint32_t start[kBuckets];
    uint32_t cur[kBuckets];
};
__device__ __forceinline__ void scatter_fused_body(const uint8_t* __restrict__ key, long long B, int chunk, int nch,
                                                   int nbk, const uint32_t* __restrict__ counts,
                                                   int32_t* __restrict__ perm, FusedLds& s, int c)
{
    uint32_t* tot = s.tot;
    uint32_t* pre = s.pre;
    uint32_t* start = s.start;
    uint32_t* cur = s.cur;
    const int t = threadIdx.x;
    const int parts = kScatThreads / nbk;  // threads (k, part): bucket k's counts over chunks part, part + parts, ...
    const int k = t % nbk, part = t / nbk;
    if (part < parts) {
        uint32_t all = 0, before = 0;
        for (int ch = part; ch < nch; ch += parts) {
            const uint32_t v = counts[(long long)ch * nbk + k];
            all += v;
            before += ch < c ? v : 0u;
        }
        tot[t] = all;
        pre[t] = before;
    }
    __syncthreads();
    uint32_t mine = 0;
    if (t < nbk) {
        uint32_t a = 0;
        for (int q = 0; q < parts; ++q) { a += tot[q * nbk + t]; mine += pre[q * nbk + t]; }
        start[t] = a;
    }
    __syncthreads();
    for (int o = 1; o < nbk; o <<= 1) {  // inclusive scan of the bucket totals, heaviest first
        const uint32_t add = (t < nbk && t >= o) ? start[t - o] : 0u;
        __syncthreads();
        if (t < nbk) start[t] += add;
        __syncthreads();
    }
    if (t < nbk) cur[t] = (t ? start[t - 1] : 0u) + mine;
    __syncthreads();
    const long long r0 = (long long)c * chunk;
    const long long r1 = r0 + chunk < B ? r0 + chunk : B;
    for (long long b = r0 + t; b < r1; b += kScatThreads) perm[atomicAdd(&cur[key[b]], 1u)] = (int32_t)b;
}

__global__ __launch_bounds__(kScatThreads) void schedule_scatter_fused_kernel(const uint8_t* __restrict__ key, long long B,
                                                                            int chunk, int nch, int nbk,
                                                                            const uint32_t* __restrict__ counts,
                                                                            int32_t* __restrict__ perm)
{
    __shared__ FusedLds s;
    scatter_fused_body(key, B, chunk, nch, nbk, counts, perm, s, blockIdx.x);
}

// Per-sector order (kSchedSectors, the sector-split launch): an X wave's work depends on the X
// sector's weight alone and a Z wave's on the Z sector's, so each sector gets its own heaviest-first
// order -- perm[0, B) for the X waves, perm[B, 2 B) for the Z waves -- from its own keys and counts
// (X and Z in one histogram pass; the scatter's first nch workgroups place X, the others Z).  P7
// fixed 20 (byte rows): 65 536 0.070 -> 0.059 ms, 262 144 0.185 -> 0.157 ms, and the split launch
// now pays at 2^19 (0.342 -> 0.294 ms) and 2^20 (0.587 -> 0.500 ms, with up to 256 fused-scatter
// chunks); P61 65 536 split +1.5 %, 131 072 -2 % (it keeps one wave per syndrome)
// (profiles/r04/cmp_sector_order_*.txt).
template <int SPLIT, bool BITS>
__global__ __launch_bounds__(kHistThreads) void schedule_hist_sec_kernel(const uint8_t* __restrict__ sX,
                                                                       const uint8_t* __restrict__ sZ, long long B,
                                                                       int mX, int mZ, int chunk, int nbk,
                                                                       uint8_t* __restrict__ keyX,
                                                                       uint32_t* __restrict__ countsX,
                                                                       uint32_t* __restrict__ zero_merge)
{
    __shared__ uint32_t hX[kBuckets], hZ[kBuckets];
    const long long nch = gridDim.x;
    uint8_t* __restrict__ keyZ = keyX + B;
    uint32_t* __restrict__ countsZ = countsX + nch * nbk;
    const int t = threadIdx.x;
    const int q = t % SPLIT;
    const long long r0 = (long long)blockIdx.x * chunk;
    const long long r1 = r0 + chunk < B ? r0 + chunk : B;
    if (t < kBuckets) hX[t] = hZ[t] = 0;
    __syncthreads();
    for (long long b = r0 + t / SPLIT; b - (t / SPLIT) < r1; b += blockDim.x / SPLIT) {
        uint32_t wx = 0, wz = 0;
        if (b < r1) {
            if constexpr (BITS) {  // mX, mZ: words per row
                const uint32_t* x = reinterpret_cast<const uint32_t*>(sX) + b * mX;
                const uint32_t* z = reinterpret_cast<const uint32_t*>(sZ) + b * mZ;
                for (int k = 0; k < mX; ++k) wx += __popc(x[k]);
                for (int k = 0; k < mZ; ++k) wz += __popc(z[k]);
            } else {
                wx = range_weight(sX, b * mX + (long long)(mX * q / SPLIT), b * mX + (long long)(mX * (q + 1) / SPLIT));
                wz = range_weight(sZ, b * mZ + (long long)(mZ * q / SPLIT), b * mZ + (long long)(mZ * (q + 1) / SPLIT));
            }
        }
#pragma unroll
        for (int o = 1; o < SPLIT; o <<= 1) {
            wx += __shfl_xor(wx, o);
            wz += __shfl_xor(wz, o);
        }
        if (q == 0 && b < r1) {
            const int kx = nbk - 1 - (int)(wx < (uint32_t)nbk - 1 ? wx : (uint32_t)nbk - 1);
            const int kz = nbk - 1 - (int)(wz < (uint32_t)nbk - 1 ? wz : (uint32_t)nbk - 1);
            keyX[b] = (uint8_t)kx;
            keyZ[b] = (uint8_t)kz;
            atomicAdd(&hX[kx], 1u);
            atomicAdd(&hZ[kz], 1u);
            if (zero_merge) zero_merge[b] = 0u;
        }
    }
    __syncthreads();
    if (t < nbk) {
        countsX[(long long)blockIdx.x * nbk + t] = hX[t];
        countsZ[(long long)blockIdx.x * nbk + t] = hZ[t];
    }
}

__global__ __launch_bounds__(kScatThreads) void schedule_scatter_sec_kernel(const uint8_t* __restrict__ keyX, long long B,
                                                                          int chunk, int nch, int nbk,
                                                                          const uint32_t* __restrict__ countsX,
                                                                          int32_t* __restrict__ perm)
{
    __shared__ FusedLds s;
    const int sec = (int)blockIdx.x >= nch ? 1 : 0;
    scatter_fused_body(keyX + sec * B, B, chunk, nch, nbk, countsX + (long long)sec * nch * nbk, perm + sec * B, s,
                       (int)blockIdx.x - sec * nch);
}

// (A cooperative single launch -- histogram, grid barrier, scatter -- was measured 4x slower than the
// two launches at P7 65 536: 0.288 vs 0.069 ms per decode call, hipLaunchCooperativeKernel's own cost;
// profiles/r03/cmp_coop_order_p7_65536.txt.)
//
// The same single launch with an ordinary launch and a software grid barrier, for at most
// kOneLaunchChunks workgroups of kScatThreads threads, and never more than the device holds at once
// (one_launch_capacity: occupancy per CU x CUs; the decoder's stream runs nothing beside them), so
// every workgroup of the grid is resident and the barrier cannot wait on one that was never scheduled;
// a larger grid takes the two-launch form.
// bar[0] counts arrivals; bar[1] departures, and the last workgroup to leave zeroes both for the next
// launch (bar comes zeroed from qec_decoder_create; graph replays reuse it the same way).
// Measured slower than the two launches it replaces (P7 65 536: 0.082 vs 0.070 ms per decode call,
// profiles/r04/cmp_one_launch_order_p7.txt): the arrival polling costs more than the launch gap.
// Kept as QEC_OPT_SCHEDULE = 4 for experiments.
constexpr int kOneLaunchChunks = 128;

__device__ __forceinline__ void grid_arrive_wait(uint32_t* bar, uint32_t nblocks)
{
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();  // this workgroup's counts before its arrival
        atomicAdd(&bar[0], 1u);
        while (__hip_atomic_load(&bar[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < nblocks)
            __builtin_amdgcn_s_sleep(2);
        __threadfence();
    }
    __syncthreads();
}

__device__ __forceinline__ void grid_depart(uint32_t* bar, uint32_t nblocks)
{
    if (threadIdx.x == 0 && atomicAdd(&bar[1], 1u) == nblocks - 1) {
        // every workgroup has passed the barrier: reset for the next launch (vector stores)
        __hip_atomic_store(&bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&bar[1], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <int MODE>  // 0: byte rows, 1: byte rows of at most kShortRows, 2: bit rows
__global__ __launch_bounds__(kScatThreads) void schedule_one_launch_kernel(const uint8_t* __restrict__ sX,
                                                                         const uint8_t* __restrict__ sZ, long long B,
                                                                         int mX, int mZ, int chunk, int nch, int nbk,
                                                                         uint8_t* __restrict__ key,
                                                                         uint32_t* __restrict__ counts,
                                                                         uint32_t* __restrict__ zero_merge,
                                                                         int32_t* __restrict__ perm, uint32_t* bar)
{
    __shared__ uint32_t h[kBuckets];
    __shared__ FusedLds s;
    if constexpr (MODE == 2)
        hist_bits_body(reinterpret_cast<const uint32_t*>(sX), reinterpret_cast<const uint32_t*>(sZ), B, mX, mZ, chunk, nbk,
                       key, counts, zero_merge, h);
    else
        hist_body<MODE == 1 ? 1 : kHistSplitLong>(sX, sZ, B, mX, mZ, chunk, nbk, key, counts, zero_merge, h);
    grid_arrive_wait(bar, (uint32_t)nch);
    scatter_fused_body(key, B, chunk, nch, nbk, counts, perm, s, blockIdx.x);
    grid_depart(bar, (uint32_t)nch);
}

// Workgroups of schedule_one_launch_kernel<MODE> the current device holds at once (occupancy per CU x
// CUs), cached per device: the software grid barrier is safe only when every workgroup of the grid is
// resident, which a smaller device or partition (fewer CUs) may not give kOneLaunchChunks.
template <int MODE>
static int one_launch_capacity()
{
    static std::atomic<int> cached[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    int cap = cached[dev].load(std::memory_order_relaxed);  // every writer stores the same value
    if (cap == 0) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, schedule_one_launch_kernel<MODE>, kScatThreads, 0) !=
                hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            per_cu = cus = 0;
        // at most one workgroup per CU is counted: the occupancy API can report one workgroup per CU more
        // than fits at some SGPR counts (MI355X_MICROARCH.md, correctness boundaries), and kOneLaunchChunks
        // is below the CU count of a whole MI355X anyway
        cap = per_cu > 0 && cus > 0 ? std::min(per_cu, 1) * cus : -1;  // -1: unknown, never take the one-launch form
        cached[dev].store(cap, std::memory_order_relaxed);
    }
    return cap;
}

// The whole order pass in one launch, for small batches (where the passes above are mostly launch
// latency): workgroup c sorts its own chunk heaviest-first in LDS and interleaves the chunks by
// rank, perm[rho * C + c] = the chunk's rank-rho syndrome.  A wave's G consecutive slots then hold
// syndromes of one rank from G chunks -- the same weight quantile, as a global sort gives them -- and
// the heaviest of every chunk come first.  Chunks have S or S - 1 syndromes (the first `rem` have S),
// so the slots rho * C + c are exactly [0, B).  No count matrix, no second pass.
constexpr int kLocalThreads = 512;
constexpr int kLocalMaxChunk = 2048;
constexpr int kLocalChunks = 128;
long long schedule_local_max_batch() { return (long long)kLocalChunks * kLocalMaxChunk; }
template <bool BITS>
__global__ __launch_bounds__(kLocalThreads) void schedule_local_kernel(const uint8_t* __restrict__ sX,
                                                                     const uint8_t* __restrict__ sZ, long long B,
                                                                     int mX, int mZ, int S, int rem, int nbk,
                                                                     int32_t* __restrict__ perm,
                                                                     uint32_t* __restrict__ zero_merge)
{
    __shared__ uint32_t h[kBuckets];
    __shared__ uint8_t key[kLocalMaxChunk];
    const int t = threadIdx.x;
    const int c = blockIdx.x, C = gridDim.x;
    const int size = c < rem ? S : S - 1;
    const long long r0 = (long long)c * (S - 1) + (c < rem ? c : rem);
    for (int k = t; k < nbk; k += blockDim.x) h[k] = 0;
    __syncthreads();
    for (int j = t; j < size; j += blockDim.x) {
        const long long b = r0 + j;
        uint32_t w = 0;
        if constexpr (BITS) {
            const uint32_t* x = reinterpret_cast<const uint32_t*>(sX) + b * mX;  // mX, mZ: words per row here
            const uint32_t* z = reinterpret_cast<const uint32_t*>(sZ) + b * mZ;
            for (int k = 0; k < mX; ++k) w += __popc(x[k]);
            for (int k = 0; k < mZ; ++k) w += __popc(z[k]);
        } else {
            w = range_weight(sX, b * mX, b * mX + mX) + range_weight(sZ, b * mZ, b * mZ + mZ);
        }
        const int bk = nbk - 1 - (int)(w < (uint32_t)nbk - 1 ? w : (uint32_t)nbk - 1);
        key[j] = (uint8_t)bk;
        atomicAdd(&h[bk], 1u);
        if (zero_merge) zero_merge[b] = 0u;
    }
    __syncthreads();
    if (t == 0) {  // exclusive scan of at most 256 buckets (heaviest first), one lane: a few hundred cycles
        uint32_t a = 0;
        for (int k = 0; k < nbk; ++k) {
            const uint32_t v = h[k];
            h[k] = a;
            a += v;
        }
    }
    __syncthreads();
    for (int j = t; j < size; j += blockDim.x) {
        const uint32_t rho = atomicAdd(&h[key[j]], 1u);
        perm[(long long)rho * C + c] = (int32_t)(r0 + j);
    }
}

// rows per chunk: at least min_chunk (one pass of the histogram workgroup), enough that there
// are at most kMaxChunks chunks
// and, below that, about kTargetChunks chunks (power-of-two sizes up to max_chunk), so a small
// batch still spreads its histogram over many workgroups (P7 65 536 at the fixed 4096 rows per chunk:
// 16 workgroups, 36 us)
static int chunk_of(long long B, int min_chunk, int max_chunk, int* nchunks)
{
    long long chunk = (B + kMaxChunks - 1) / kMaxChunks;
    long long want = min_chunk;
    while (want < max_chunk && want * kTargetChunks < B) want *= 2;
    if (chunk < want) chunk = want;
    *nchunks = (int)((B + chunk - 1) / chunk);
    return (int)chunk;
}

// B <= kMaxChunks * kMaxChunk syndromes per ordered launch (4 M)
long long schedule_max_batch() { return (long long)kMaxChunks * kMaxChunk; }

// whether a batch of B syndromes that asks for it gets the per-sector order (its chunks fit the fused scatter)
bool schedule_sector_order(long long B, bool sbits, int mX, int mZ)
{
    if (!kSchedSectors || B <= 1 || B > schedule_max_batch()) return false;
    const bool shortrows = sbits || mX + mZ <= kShortRows;
    int nch = 0;
    chunk_of(B, 256, shortrows ? 4 * kHistThreads : 512, &nch);
    return nch <= kMaxFusedChunks;
}

// workspace layout: perm [2 B] i32 (the per-sector order takes both halves), counts [chunks][256] u32
// (per-sector: X then Z, [nch][nbk] each, at most kMaxFusedChunks chunks), totals [256] u32, key [2 B] u8
static size_t perm_bytes(long long B) { return ((size_t)2 * B * sizeof(int32_t) + 255) & ~(size_t)255; }

size_t schedule_workspace_bytes(long long B, int, int)
{
    return perm_bytes(B) + (size_t)kMaxChunks * kBuckets * 4 + kBuckets * 4 + 2 * B + 64;
}

// Fills the workspace (schedule_workspace_bytes bytes) and returns in *perm_out the
// heaviest-first order of the batch.  zero_merge (nullable): B words the hist pass zeroes on
// the way (the sector-split decode merges its two sectors' flags there, bp_decode.hip).
// want_sectors (sector-split waves or sector launches): the per-sector order where the fused scatter
// takes the batch (*sectors_out = true: 2 B entries, the Z waves' order from perm[B]).  bar (nullable): the handle's two zeroed grid-barrier words
// (schedule_one_launch_kernel).
int launch_schedule(const uint8_t* sX, const uint8_t* sZ, bool sbits, long long B, int mX, int mZ, void* ws,
                    uint32_t* zero_merge, bool want_sectors, int32_t** perm_out, bool* sectors_out, hipStream_t st,
                    int method, uint32_t* bar)
{
    *sectors_out = false;
    if (B > schedule_max_batch()) return fail(QEC_ERR_ARG, "schedule: batch too large to order");
    const bool shortrows = sbits || mX + mZ <= kShortRows;
    if (method == QEC_ORDER_LOCAL && shortrows && B <= schedule_local_max_batch()) {
        // one launch: C chunks of about B / C syndromes (at most kLocalMaxChunk), sorted locally and
        // interleaved by rank (schedule_local_kernel)
        int C = kLocalChunks;
        while (C > 1 && (B + C - 1) / C < 256) C /= 2;
        const long long S = (B + C - 1) / C;
        const int rem = (int)(B - (S - 1) * C);
        const int nbk = mX + mZ + 1 < kBuckets ? mX + mZ + 1 : kBuckets;
        int32_t* perm = reinterpret_cast<int32_t*>(ws);
        *perm_out = perm;
        const int threads = S >= kLocalThreads ? kLocalThreads : (int)((S + 63) / 64 * 64);
        if (sbits)
            hipLaunchKernelGGL(schedule_local_kernel<true>, dim3(C), dim3(threads), 0, st, sX, sZ, B, (mX + 31) / 32,
                               (mZ + 31) / 32, (int)S, rem, nbk, perm, zero_merge);
        else
            hipLaunchKernelGGL(schedule_local_kernel<false>, dim3(C), dim3(threads), 0, st, sX, sZ, B, mX, mZ, (int)S,
                               rem, nbk, perm, zero_merge);
        const hipError_t err = hipGetLastError();
        if (err != hipSuccess) return fail(QEC_ERR_HIP, std::string("schedule launch: ") + hipGetErrorString(err));
        return QEC_OK;
    }
    int nch = 0;
    // short rows: 4096 syndromes per chunk (four per thread): the offsets and scatter passes then
    // handle a quarter of the chunks (P7 2^20: order pass 60 -> 51 us, profiles/r02/hist_ab_r02s3zj.txt;
    // staging the rows through LDS did not speed the histogram up)
    const int split = shortrows ? 1 : kHistSplitLong;
    const int chunk = chunk_of(B, 256, shortrows ? 4 * kHistThreads : 512, &nch);
    // histogram workgroup: one pass over its chunk when the chunk is small (256 .. 1024 threads)
    int hthreads = chunk * split;
    hthreads = hthreads < 256 ? 256 : hthreads > kHistThreads ? kHistThreads : (hthreads + 63) / 64 * 64;
    uint8_t* p = static_cast<uint8_t*>(ws);
    int32_t* perm = reinterpret_cast<int32_t*>(p);
    uint32_t* counts = reinterpret_cast<uint32_t*>(p + perm_bytes(B));
    uint32_t* totals = counts + (size_t)kMaxChunks * kBuckets;
    uint8_t* key = reinterpret_cast<uint8_t*>(totals + kBuckets);
    *perm_out = perm;
    const bool fused = nch <= kMaxFusedChunks;
    // buckets: weights 0 .. mX + mZ (fused pass), 256 for the separate offsets / scatter passes
    int nbk = kBuckets;
    if (fused && mX + mZ + 1 < kBuckets) nbk = mX + mZ + 1 < 32 ? 32 : mX + mZ + 1;
    if (kSchedSectors && method == QEC_ORDER_GLOBAL && want_sectors && fused) {
        const int nbs = std::max(32, std::min(kBuckets, std::max(mX, mZ) + 1));  // sector weights 0 .. max(mX, mZ)
        if (sbits)
            hipLaunchKernelGGL((schedule_hist_sec_kernel<1, true>), dim3(nch), dim3(hthreads), 0, st, sX, sZ, B, (mX + 31) / 32,
                               (mZ + 31) / 32, chunk, nbs, key, counts, zero_merge);
        else if (shortrows)
            hipLaunchKernelGGL((schedule_hist_sec_kernel<1, false>), dim3(nch), dim3(hthreads), 0, st, sX, sZ, B, mX, mZ, chunk,
                               nbs, key, counts, zero_merge);
        else
            hipLaunchKernelGGL((schedule_hist_sec_kernel<kHistSplitLong, false>), dim3(nch), dim3(hthreads), 0, st, sX, sZ, B,
                               mX, mZ, chunk, nbs, key, counts, zero_merge);
        hipLaunchKernelGGL(schedule_scatter_sec_kernel, dim3(2 * nch), dim3(kScatThreads), 0, st, key, B, chunk, nch, nbs,
                           counts, perm);
        const hipError_t err = hipGetLastError();
        if (err != hipSuccess) return fail(QEC_ERR_HIP, std::string("schedule launch: ") + hipGetErrorString(err));
        *sectors_out = true;
        return QEC_OK;
    }
    const int one_cap = method != QEC_ORDER_ONE_LAUNCH ? 0
                        : sbits                       ? one_launch_capacity<2>()
                        : shortrows                   ? one_launch_capacity<1>()
                                                      : one_launch_capacity<0>();
    if (method == QEC_ORDER_ONE_LAUNCH && fused && bar != nullptr && nch <= kOneLaunchChunks && nch <= one_cap) {
        // histogram, grid barrier, offsets and scatter in one launch (schedule_one_launch_kernel)
        if (sbits)
            hipLaunchKernelGGL(schedule_one_launch_kernel<2>, dim3(nch), dim3(kScatThreads), 0, st, sX, sZ, B,
                               (mX + 31) / 32, (mZ + 31) / 32, chunk, nch, nbk, key, counts, zero_merge, perm, bar);
        else if (shortrows)
            hipLaunchKernelGGL(schedule_one_launch_kernel<1>, dim3(nch), dim3(kScatThreads), 0, st, sX, sZ, B, mX, mZ,
                               chunk, nch, nbk, key, counts, zero_merge, perm, bar);
        else
            hipLaunchKernelGGL(schedule_one_launch_kernel<0>, dim3(nch), dim3(kScatThreads), 0, st, sX, sZ, B, mX, mZ,
                               chunk, nch, nbk, key, counts, zero_merge, perm, bar);
        const hipError_t err = hipGetLastError();
        if (err != hipSuccess) return fail(QEC_ERR_HIP, std::string("schedule launch: ") + hipGetErrorString(err));
        return QEC_OK;
    }
    if (sbits)
        hipLaunchKernelGGL(schedule_hist_bits_kernel, dim3(nch), dim3(hthreads), 0, st,
                           reinterpret_cast<const uint32_t*>(sX), reinterpret_cast<const uint32_t*>(sZ), B, (mX + 31) / 32,
                           (mZ + 31) / 32, chunk, nbk, key, counts, zero_merge);
    else if (shortrows)
        hipLaunchKernelGGL(schedule_hist_kernel<1>, dim3(nch), dim3(hthreads), 0, st, sX, sZ, B, mX, mZ, chunk, nbk, key,
                           counts, zero_merge);
    else
        hipLaunchKernelGGL(schedule_hist_kernel<kHistSplitLong>, dim3(nch), dim3(hthreads), 0, st, sX, sZ, B, mX, mZ,
                           chunk, nbk, key, counts, zero_merge);
    if (fused) {
        hipLaunchKernelGGL(schedule_scatter_fused_kernel, dim3(nch), dim3(kScatThreads), 0, st, key, B, chunk, nch, nbk,
                           counts, perm);
    } else {
        hipLaunchKernelGGL(schedule_offsets_kernel, dim3(kBuckets), dim3(kScanThreads), 0, st, nch, counts, totals);
        hipLaunchKernelGGL(schedule_scatter_kernel, dim3(nch), dim3(kScatThreads), 0, st, key, B, chunk, counts, totals,
                           perm);
    }
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) return fail(QEC_ERR_HIP, std::string("schedule launch: ") + hipGetErrorString(err));
    return QEC_OK;
}

}  // namespace qec
