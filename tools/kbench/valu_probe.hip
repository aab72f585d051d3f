// VALU issue-rate probe for the instruction mix of the BP kernels (gfx950).
// Independent chains (NCH per lane) of one operation, 8 waves per SIMD; each wave
// times itself with s_memtime (shader-clock ticks), so the result is SIMD-cycles
// per wave-instruction independent of the clock the part actually ran at.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize tools/kbench/valu_probe.hip -o build/valu_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#pragma clang fp contract(off)

typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int kIters = 8192;

__device__ __forceinline__ f2 pk_mul(f2 a, f2 b)
{
    f2 r;
    asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c)
{
    f2 r;
    asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ f2 pk_add(f2 a, f2 b)
{
    f2 r;
    asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float mul(float a, float b)
{
    float r;
    asm volatile("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float rcp(float a)
{
    float r;
    asm volatile("v_rcp_f32 %0, %1" : "=v"(r) : "v"(a));
    return r;
}

__device__ __forceinline__ float fma3(float a, float b, float c)
{
    float r;
    asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float add(float a, float b)
{
    float r;
    asm volatile("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float dscale(float a, float b)
{
    float r;
    unsigned long long sc;
    asm volatile("v_div_scale_f32 %0, %1, %2, %2, %3" : "=v"(r), "=s"(sc) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float dfixup(float a, float b, float c)
{
    float r;
    asm volatile("v_div_fixup_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float dfmas(float a, float b, float c)
{
    float r;
    asm volatile("s_mov_b64 vcc, 0\n\tv_div_fmas_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c) : "vcc");
    return r;
}

__device__ __forceinline__ float bperm(float a, int addr)
{
    return __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(a)));
}

// OP 0: v_mul_f32, 1: v_pk_mul_f32 (2 fp32 products / lane), 2: v_rcp_f32,
// 3: IEEE fp32 division as hipcc emits it (11 instructions), counted per division,
// 4: v_fma_f32, 5: v_add_f32, 6: v_div_scale_f32, 7: v_div_fixup_f32,
// 8: v_div_fmas_f32 (+ one s_mov_b64 vcc each), 9: ds_bpermute_b32, 10: 1 ds_bpermute + NCH-1 v_mul,
// 11: v_pk_fma_f32, 12: v_pk_add_f32, 13: v_mul / v_rcp alternating, 14: 1 v_rcp per 4 v_mul.
template <int OP, int NCH>
__global__ __launch_bounds__(256) void probe(long long* cycles, float a)
{
    float x[NCH];
    f2 y[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        x[c] = 0.75f + 0.001f * c + 1e-5f * threadIdx.x;
        y[c] = f2{x[c], x[c] + 0.5f};
    }
    const f2 a2 = f2{a, a};
    __builtin_amdgcn_s_waitcnt(0);
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            if (OP == 0) x[c] = mul(x[c], a);
            if (OP == 1) y[c] = pk_mul(y[c], a2);
            if (OP == 2) x[c] = rcp(x[c]);
            if (OP == 3) x[c] = a / x[c];
            if (OP == 4) x[c] = fma3(x[c], a, 0.0001f);
            if (OP == 5) x[c] = add(x[c], a);
            if (OP == 6) x[c] = dscale(x[c], a);
            if (OP == 7) x[c] = dfixup(x[c], a, 0.75f);
            if (OP == 8) x[c] = dfmas(x[c], a, 0.0001f);
            if (OP == 9) x[c] = bperm(x[c], (int)((threadIdx.x * 4 + 4 * (c + 1)) & 255));
            if (OP == 10) x[c] = c == 0 ? bperm(x[c], (int)((threadIdx.x * 4 + 4) & 255)) : mul(x[c], a);
            if (OP == 11) y[c] = pk_fma(y[c], a2, f2{0.0001f, 0.0002f});
            if (OP == 12) y[c] = pk_add(y[c], a2);
            // half the chains v_mul_f32, half v_rcp_f32 (does the transcendental overlap plain VALU?)
            if (OP == 13) x[c] = (c & 1) ? rcp(x[c]) : mul(x[c], a);
            // 1 v_rcp_f32 per 4 v_mul_f32 (about the division mix of the var pass)
            if (OP == 14) x[c] = (c % 5 == 0) ? rcp(x[c]) : mul(x[c], a);
            if (OP == 15) x[c] = __int_as_float(__float_as_int(x[c]) ^ (int)(threadIdx.x + c));
            if (OP == 16) x[c] = __uint_as_float(min(__float_as_uint(x[c]) + 1u, 0x3F800000u + (uint32_t)c));
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.0f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) s += x[c] + y[c].x + y[c].y;
    if ((threadIdx.x & 63) == 0) cycles[blockIdx.x * 4 + (threadIdx.x >> 6)] = (t1 - t0) + (s == 1.2345f);
}

static double g_mhz = 0;  // s_memtime ticks per microsecond of the last timed launch
static double g_ev = 0;   // the last timed launch by HIP events: SIMD-cycles per wave-instruction at 2.4 GHz

static int cus_g = 256;
template <int OP, int NCH>
static double run(long long* d, int blocks, std::vector<long long>& h, int wps = 8)
{
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((probe<OP, NCH>), dim3(blocks), dim3(256), 0, 0, d, 0.9999f);
    hipEventRecord(e0);
    hipLaunchKernelGGL((probe<OP, NCH>), dim3(blocks), dim3(256), 0, 0, d, 0.9999f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipDeviceSynchronize();
    hipMemcpy(h.data(), d, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
    double sum = 0;
    const size_t nw = (size_t)blocks * 4;
    for (size_t k = 0; k < nw; ++k) sum += (double)h[k];
    const double mean_wave_cycles = sum / nw;
    long long mx = 0;
    for (size_t k = 0; k < nw; ++k) mx = h[k] > mx ? h[k] : mx;
    g_mhz = mx / (ms * 1e3);  // the longest wave spans ~the whole launch
    // launch time (events, includes launch overhead and the wave start/finish ramp) in 2.4 GHz
    // cycles over the instructions each SIMD issued: an upper bound on the per-instruction cost
    g_ev = (ms * 1e-3 * 2.4e9) / ((double)wps * kIters * NCH) * ((double)cus_g * 4 * wps / ((double)blocks * 4));
    // 8 waves share each SIMD for the whole run: SIMD-cycles per wave-instruction
    return mean_wave_cycles / ((double)wps * kIters * NCH);
}

// Throughput by HIP events alone, on an oversubscribed grid (32 waves per SIMD requested, 8 resident
// at a time): wave-instructions retired per SIMD per 2.4 GHz cycle, independent of how the issue
// arbiter shares the SIMD between its resident waves (s_memtime per wave assumes fair sharing).
template <int OP, int NCH>
static double tp(long long* d, int cus, int gens = 4)
{
    const int blocks = cus * 8 * gens;
    long long* big = nullptr;
    hipMalloc(&big, sizeof(long long) * blocks * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL((probe<OP, NCH>), dim3(blocks), dim3(256), 0, 0, big, 0.9999f);
    hipEventRecord(e0);
    hipLaunchKernelGGL((probe<OP, NCH>), dim3(blocks), dim3(256), 0, 0, big, 0.9999f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipFree(big);
    const double instrs_per_simd = (double)blocks * 4 * kIters * NCH / (cus * 4.0);
    return ms * 1e-3 * 2.4e9 / instrs_per_simd;
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    cus_g = cus;
    const int blocks = cus * 8;  // 32 waves per CU = 8 per SIMD
    long long* d = nullptr;
    hipMalloc(&d, sizeof(long long) * blocks * 4);
    std::vector<long long> h((size_t)blocks * 4);
    printf("{\"cus\": %d, \"waves_per_simd\": 8", cus);
    printf(", \"v_mul_f32 x8\": %.3f", run<0, 8>(d, blocks, h));
    printf(", \"v_mul_f32 x8 [events @2.4GHz]\": %.3f", g_ev);
    printf(", \"v_mul_f32 x16\": %.3f", run<0, 16>(d, blocks, h));
    printf(", \"v_pk_mul_f32 x8\": %.3f", run<1, 8>(d, blocks, h));
    printf(", \"v_pk_mul_f32 x8 [events @2.4GHz]\": %.3f", g_ev);
    printf(", \"v_pk_mul_f32 x16\": %.3f", run<1, 16>(d, blocks, h));
    printf(", \"v_rcp_f32 x8\": %.3f", run<2, 8>(d, blocks, h));
    printf(", \"v_rcp_f32 x8 [events @2.4GHz]\": %.3f", g_ev);
    printf(", \"fp32 division x8\": %.3f", run<3, 8>(d, blocks, h));
    printf(", \"memtime_ticks_per_us\": %.1f", g_mhz);
    printf(", \"v_fma_f32 x8\": %.3f", run<4, 8>(d, blocks, h));
    printf(", \"v_fma_f32 x8 [events @2.4GHz]\": %.3f", g_ev);
    printf(", \"v_add_f32 x8\": %.3f", run<5, 8>(d, blocks, h));
    printf(", \"v_div_scale_f32 x8\": %.3f", run<6, 8>(d, blocks, h));
    printf(", \"v_div_fixup_f32 x8\": %.3f", run<7, 8>(d, blocks, h));
    printf(", \"v_div_fmas_f32+s_mov x8\": %.3f", run<8, 8>(d, blocks, h));
    // latency: one dependent chain per wave, 1 / 2 / 4 / 8 waves per SIMD
    for (int wps : {1, 2, 4, 8}) {
        printf(", \"v_mul_f32 x1 @%dw\": %.3f", wps, run<0, 1>(d, cus * wps, h, wps));
        printf(", \"v_mul_f32 x2 @%dw\": %.3f", wps, run<0, 2>(d, cus * wps, h, wps));
    }
    printf(", \"v_fma_f32 x1 @1w\": %.3f", run<4, 1>(d, cus, h, 1));
    printf(", \"v_rcp_f32 x1 @1w\": %.3f", run<2, 1>(d, cus, h, 1));
    printf(", \"fp32 division x1 @1w\": %.3f", run<3, 1>(d, cus, h, 1));
    printf(", \"fp32 division x4 @5w\": %.3f", run<3, 4>(d, cus * 5, h, 5));
    printf(", \"ds_bpermute x8 @8w\": %.3f", run<9, 8>(d, blocks, h));
    printf(", \"ds_bpermute x8 @8w [events @2.4GHz]\": %.3f", g_ev);
    printf(", \"ds_bpermute x1 @1w\": %.3f", run<9, 1>(d, cus, h, 1));
    // overlap of LDS permutes with VALU: 1 ds_bpermute chain + 14 v_mul chains per step
    printf(", \"bperm1+mul14 @5w (per step)\": %.3f", 15.0 * run<10, 15>(d, cus * 5, h, 5));
    printf(", \"mul14 @5w (per step)\": %.3f", 14.0 * run<0, 14>(d, cus * 5, h, 5));
    printf(", \"bperm1 @5w (per step)\": %.3f", run<9, 1>(d, cus * 5, h, 5));
    printf(", \"bperm8 @5w (per instr)\": %.3f", run<9, 8>(d, cus * 5, h, 5));
    printf(", \"v_pk_fma_f32 x8\": %.3f", run<11, 8>(d, blocks, h));
    printf(", \"v_pk_fma_f32 x8 [events @2.4GHz]\": %.3f", g_ev);
    printf(", \"v_pk_add_f32 x8\": %.3f", run<12, 8>(d, blocks, h));
    printf(", \"v_mul_f32 x8 @5w\": %.3f", run<0, 8>(d, cus * 5, h, 5));
    printf(", \"v_mul_f32 x8 @5w [events @2.4GHz]\": %.3f", g_ev);
    printf(", \"v_pk_mul_f32 x8 @5w\": %.3f", run<1, 8>(d, cus * 5, h, 5));
    printf(", \"v_rcp_f32 x8 @5w\": %.3f", run<2, 8>(d, cus * 5, h, 5));
    printf(", \"mul/rcp alternating x8 (per instr)\": %.3f", run<13, 8>(d, blocks, h));
    printf(", \"1 rcp + 4 mul x10 (per instr)\": %.3f", run<14, 10>(d, blocks, h));
    printf(", \"v_pk_mul_f32 x1 @1w\": %.3f", run<1, 1>(d, cus, h, 1));
    printf(", \"v_mul_f32 x8 @1w\": %.3f", run<0, 8>(d, cus, h, 1));
    printf(", \"v_pk_mul_f32 x8 @1w\": %.3f", run<1, 8>(d, cus, h, 1));
    printf(", \"v_rcp_f32 x8 @1w\": %.3f", run<2, 8>(d, cus, h, 1));
    printf(", \"throughput\": {\"unit\": \"2.4 GHz cycles per wave-instruction per SIMD (events, 32 waves/SIMD requested)\"");
    printf(", \"v_mul_f32 x8\": %.3f", tp<0, 8>(d, cus));
    printf(", \"v_mul_f32 x16\": %.3f", tp<0, 16>(d, cus));
    printf(", \"v_add_f32 x8\": %.3f", tp<5, 8>(d, cus));
    printf(", \"v_fma_f32 x8\": %.3f", tp<4, 8>(d, cus));
    printf(", \"v_pk_mul_f32 x8\": %.3f", tp<1, 8>(d, cus));
    printf(", \"v_pk_fma_f32 x8\": %.3f", tp<11, 8>(d, cus));
    printf(", \"v_rcp_f32 x8\": %.3f", tp<2, 8>(d, cus));
    printf(", \"v_xor_b32 x8\": %.3f", tp<15, 8>(d, cus));
    printf(", \"v_add_u32+v_min_u32 x8 (per pair)\": %.3f", tp<16, 8>(d, cus));
    printf(", \"1 rcp + 4 mul x10 (per instr)\": %.3f", tp<14, 10>(d, cus));
    printf(", \"ds_bpermute x8\": %.3f", tp<9, 8>(d, cus));
    printf(", \"1 bpermute + 14 mul (per instr)\": %.3f", tp<10, 15>(d, cus));
    printf(", \"fp32 division x8 (per division)\": %.3f", tp<3, 8>(d, cus));
    printf(", \"v_mul_f32 x8, 1 gen\": %.3f", tp<0, 8>(d, cus, 1));
    printf(", \"v_mul_f32 x8, 16 gens\": %.3f}", tp<0, 8>(d, cus, 16));
    printf(", \"unit\": \"SIMD-cycles per wave-instruction (s_memtime)\"}\n");
    hipFree(d);
    return 0;
}
