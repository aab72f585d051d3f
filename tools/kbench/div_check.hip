// Exhaustive / randomised check of a 6-instruction correctly rounded fp32 division for the
// operand range bp_decode.hip's short division is guarded to (gfx950):
//   y0 = rcp(b); e = fma(-b, y0, 1); y1 = fma(e, y0, y0)        (refined reciprocal)
//   q0 = a * y1; r = fma(-b, q0, a); q1 = fma(r, y1, q0)        (one residual correction)
// Markstein's theorem: if y1 = RN(1/b) and q0 is within one ulp of a/b, then q1 = RN(a/b)
// (no underflow/overflow on the way).  Part 1 checks y1 == RN(1/b) for EVERY b in [2^-98, 2]
// (all significands, every exponent); part 2 compares q1 with the IEEE quotient on random
// (a, b) pairs of the guarded domain (a = +0 or 2^-98 <= a <= b) and on near-midpoint pairs.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/kbench/div_check.hip -o build/div_check
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#pragma clang fp contract(off)

__device__ __forceinline__ float rcp_refined(float b)
{
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y0, 1.0f);
    return __builtin_fmaf(e, y0, y0);
}

__device__ __forceinline__ float div6(float a, float b)
{
    const float y1 = rcp_refined(b);
    const float q0 = a * y1;
    const float r = __builtin_fmaf(-b, q0, a);
    return __builtin_fmaf(r, y1, q0);
}

// 8-instruction form used today (bp_decode.hip div_short)
__device__ __forceinline__ float div8(float a, float b)
{
    float r = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, r, 1.0f);
    r = __builtin_fmaf(e, r, r);
    float q = a * r;
    const float e2 = __builtin_fmaf(-b, q, a);
    q = __builtin_fmaf(e2, r, q);
    const float e3 = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(e3, r, q);
}

// part 1: thread per significand, loop over exponents 2^-98 .. 2^0 (b < 2)
__global__ void recip_kernel(unsigned long long* bad, unsigned int* first)
{
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= (1u << 23)) return;
    unsigned long long nb = 0;
    for (int ex = -98; ex <= 0; ++ex) {
        const float b = __uint_as_float(((uint32_t)(ex + 127) << 23) | m);
        const float y1 = rcp_refined(b);
        const float ref = 1.0f / b;
        if (__float_as_uint(y1) != __float_as_uint(ref)) {
            ++nb;
            atomicMin(first, __float_as_uint(b));
        }
    }
    if (nb) atomicAdd(bad, nb);
}

__device__ __forceinline__ uint32_t hash32(uint64_t x)
{
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return (uint32_t)x;
}

// part 2: random pairs; mode 0 uniform bit patterns in the domain, mode 1 near midpoints
__global__ void pair_kernel(uint64_t seed, int per_thread, int mode, unsigned long long* bad6,
                            unsigned long long* bad8, unsigned int* ex_a, unsigned int* ex_b)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long n6 = 0, n8 = 0;
    for (int k = 0; k < per_thread; ++k) {
        const uint64_t c = (t * per_thread + k) * 4 + seed;
        // b: exponent in [-98, 0], any significand
        const uint32_t hb = hash32(c), ha = hash32(c + 1), hq = hash32(c + 2);
        const int eb = -98 + (int)(hb % 99u);
        const float b = __uint_as_float(((uint32_t)(eb + 127) << 23) | (hb >> 9));
        float a;
        if (mode == 0) {
            // a <= b: exponent in [-98, eb], random significand, clamp to b; 1/64 of the time +0
            const int ea = -98 + (int)(ha % (uint32_t)(eb + 99));
            a = __uint_as_float(((uint32_t)(ea + 127) << 23) | (hq >> 9));
            if (a > b) a = b;
            if ((ha & 63u) == 0) a = 0.0f;
        } else {
            // a = b * q for a random q in [2^-60, 1), perturbed by a few ulps: quotients close to
            // rounding boundaries
            const float q = __uint_as_float(((uint32_t)(127 - 1 - (int)(ha % 60u)) << 23) | (hq >> 9));
            a = b * q;
            const int d = (int)((ha >> 8) & 7u) - 3;
            a = __uint_as_float(__float_as_uint(a) + d);
            if (!(a >= 0x1p-98f) || a > b) continue;
        }
        const float ref = a / b;
        if (__float_as_uint(div6(a, b)) != __float_as_uint(ref)) {
            ++n6;
            *ex_a = __float_as_uint(a);
            *ex_b = __float_as_uint(b);
        }
        if (__float_as_uint(div8(a, b)) != __float_as_uint(ref)) ++n8;
    }
    if (n6) atomicAdd(bad6, n6);
    if (n8) atomicAdd(bad8, n8);
}

int main(int argc, char** argv)
{
    unsigned long long* d;
    unsigned int* u;
    hipMalloc(&d, 4 * sizeof(unsigned long long));
    hipMalloc(&u, 4 * sizeof(unsigned int));
    hipMemset(d, 0, 4 * sizeof(unsigned long long));
    unsigned int init[4] = {0xFFFFFFFFu, 0, 0, 0};
    hipMemcpy(u, init, sizeof init, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(recip_kernel, dim3((1u << 23) / 256), dim3(256), 0, 0, d, u);
    hipDeviceSynchronize();
    unsigned long long h[4];
    unsigned int hu[4];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    hipMemcpy(hu, u, sizeof hu, hipMemcpyDeviceToHost);
    printf("{\"recip_checked\": %llu, \"recip_mismatch\": %llu, \"recip_first_bad_b\": \"0x%08x\"",
           (unsigned long long)(1u << 23) * 99ull, h[0], hu[0]);
    const int per = argc > 1 ? atoi(argv[1]) : 256;
    const unsigned blocks = 65536;
    for (int mode = 0; mode < 2; ++mode) {
        hipMemset(d, 0, 4 * sizeof(unsigned long long));
        hipLaunchKernelGGL(pair_kernel, dim3(blocks), dim3(256), 0, 0, (uint64_t)(mode + 1) << 40, per, mode, d, d + 1,
                           u + 1, u + 2);
        hipDeviceSynchronize();
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        hipMemcpy(hu, u, sizeof hu, hipMemcpyDeviceToHost);
        printf(", \"pairs_mode%d\": %llu, \"div6_mismatch_mode%d\": %llu, \"div8_mismatch_mode%d\": %llu, "
               "\"div6_example_mode%d\": [\"0x%08x\", \"0x%08x\"]",
               mode, (unsigned long long)blocks * 256ull * per, mode, h[0], mode, h[1], mode, hu[1], hu[2]);
    }
    printf("}\n");
    return 0;
}
