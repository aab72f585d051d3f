// Exhaustive check of a 4-instruction fp32 division candidate on gfx950 (experiment):
//   y0 = rcp(d); q0 = n * y0; r = fma(-d, q0, n); q1 = fma(r, y0, q0)
// i.e. bp_decode.hip's short division (div_short) without the reciprocal refinement y1 = RN(1/d).
// Markstein's theorem needs y = RN(1/d); with the raw v_rcp_f32 (about 1 ulp) it gives no guarantee,
// so this runs the candidate against the IEEE quotient n / d on EVERY pair of significands (n, d in
// [1, 2): 2^46 pairs; scaling n or d by a power of two scales q0, r and q1 exactly while everything
// stays normal, so these pairs stand for the whole normal domain of the scaled folds), after
// checking that v_rcp_f32 itself is exponent-independent there (rcp(m 2^e) == rcp(m) 2^-e for every
// significand m and e in [-100, 40], the guarded and the scaled domains).  Prints one JSON line; any mismatch rules the candidate out.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/kbench/div4_check.hip -o tools/kbench/div4_check
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#pragma clang fp contract(off)

__device__ __forceinline__ float div4(float n, float d)
{
    const float y0 = __builtin_amdgcn_rcpf(d);
    const float q0 = n * y0;
    const float r = __builtin_fmaf(-d, q0, n);
    return __builtin_fmaf(r, y0, q0);
}

// part 1: thread per significand m of d; rcp(m 2^e) against rcp(m) 2^-e for e in [-100, 40]
__global__ void rcp_scale_kernel(unsigned long long* bad)
{
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= (1u << 23)) return;
    const float d1 = __uint_as_float((127u << 23) | m);
    const uint32_t y1 = __float_as_uint(__builtin_amdgcn_rcpf(d1));
    unsigned long long nb = 0;
    for (int e = -100; e <= 40; ++e) {
        const float d = __uint_as_float(((uint32_t)(127 + e) << 23) | m);
        const uint32_t y = __float_as_uint(__builtin_amdgcn_rcpf(d));
        // y1 2^-e: the exponent field moves by -e (y1 is in (0.5, 1], its scaled value stays normal)
        const uint32_t want = y1 - ((uint32_t)e << 23);
        nb += y != want;
    }
    if (nb) atomicAdd(bad, nb);
}

// part 2: thread per significand j of d, n's significands i in [i0, i0 + span)
__global__ void pair_kernel(uint32_t i0, uint32_t span, unsigned long long* bad, unsigned long long* first)
{
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= (1u << 23)) return;
    const float d = __uint_as_float((127u << 23) | j);
    unsigned long long nb = 0;
    for (uint32_t i = i0; i < i0 + span; ++i) {
        const float n = __uint_as_float((127u << 23) | i);
        const float ref = n / d;  // IEEE (div_scale / div_fmas / div_fixup)
        const float got = div4(n, d);
        if (__float_as_uint(ref) != __float_as_uint(got)) {
            ++nb;
            atomicMin(first, ((unsigned long long)i << 32) | j);
        }
    }
    if (nb) atomicAdd(bad, nb);
}

int main(int argc, char** argv)
{
    const int launches = argc > 1 ? atoi(argv[1]) : 256;  // n-significand slices (2^23 / launches each)
    unsigned long long *bad = nullptr, *first = nullptr;
    if (hipMalloc(&bad, 2 * sizeof(unsigned long long)) != hipSuccess || hipMalloc(&first, sizeof(unsigned long long)) != hipSuccess)
        return 1;
    (void)hipMemset(bad, 0, 2 * sizeof(unsigned long long));
    (void)hipMemset(first, 0xFF, sizeof(unsigned long long));
    hipLaunchKernelGGL(rcp_scale_kernel, dim3((1u << 23) / 256), dim3(256), 0, 0, bad);
    const uint32_t span = (1u << 23) / (uint32_t)launches;
    for (int L = 0; L < launches; ++L) {
        hipLaunchKernelGGL(pair_kernel, dim3((1u << 23) / 256), dim3(256), 0, 0, (uint32_t)L * span, span, bad + 1, first);
        if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); return 1; }
        if (L % 16 == 15) { fprintf(stderr, "slice %d/%d\n", L + 1, launches); fflush(stderr); }
    }
    unsigned long long h[2], f;
    (void)hipMemcpy(h, bad, sizeof h, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&f, first, sizeof f, hipMemcpyDeviceToHost);
    printf("{\"rcp_scale_mismatches\": %llu, \"pairs\": %llu, \"pair_mismatches\": %llu, \"first_i\": %lld, \"first_j\": %lld}\n",
           h[0], (unsigned long long)span * launches * (1ull << 23), h[1], h[1] ? (long long)(f >> 32) : -1LL,
           h[1] ? (long long)(f & 0xFFFFFFFFu) : -1LL);
    return 0;
}
