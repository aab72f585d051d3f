// Cycle cost of the 61-lane ring rotation as a pull (ds_bpermute_b32: lane j reads lane (j + s) mod 61)
// and as a push (ds_permute_b32: lane j writes lane (j + u) mod 61, the same rotation for u = 61 - s),
// per shift, at full occupancy.  Question: do the wrapped 32-lane halves of a pull (s >= 30) conflict
// on the LDS banks while the push of the same rotation (u = 61 - s <= 31) does not?
//   hipcc --offload-arch=gfx950 -O3 -o tools/kbench/perm_probe tools/kbench/perm_probe.hip
//   tools/kbench/perm_probe  -> one line per shift: pull_ms push_ms
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kChains = 8;

template <bool PUSH>
__global__ __launch_bounds__(256) void rotate_kernel(float* out, int s, int iters)
{
    const int lane = threadIdx.x & 63;
    int t = lane + s;
    if (t >= 61) t -= 61;
    if (lane >= 61) t = lane;  // the idle lanes address themselves
    const int addr = t * 4;
    int v[kChains];
#pragma unroll
    for (int c = 0; c < kChains; ++c) v[c] = lane * kChains + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < kChains; ++c)
            v[c] = PUSH ? __builtin_amdgcn_ds_permute(addr, v[c]) : __builtin_amdgcn_ds_bpermute(addr, v[c]);
    }
    int acc = 0;
#pragma unroll
    for (int c = 0; c < kChains; ++c) acc ^= v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)acc;
}

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                       \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

int main(int argc, char** argv)
{
    const int iters = argc > 1 ? std::atoi(argv[1]) : 2048;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int blocks = prop.multiProcessorCount * 8;  // 8 blocks of 4 waves per CU: 8 waves per SIMD
    float* out = nullptr;
    CK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(float)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(rotate_kernel<false>, dim3(blocks), dim3(256), 0, 0, out, 1, iters);
    hipLaunchKernelGGL(rotate_kernel<true>, dim3(blocks), dim3(256), 0, 0, out, 1, iters);
    CK(hipDeviceSynchronize());
    const double insts = (double)blocks * 4 * iters * kChains;  // wave-instructions per launch
    std::printf("# shift pull_ms push_ms pull_cyc push_cyc (LDS cycles per wave-instruction per CU at %d MHz)\n",
                prop.clockRate / 1000);
    for (int s = 0; s <= 60; ++s) {
        float ms[2];
        for (int k = 0; k < 2; ++k) {
            const int sh = k ? (61 - s) % 61 : s;  // the same rotation as a push
            CK(hipEventRecord(e0, 0));
            for (int r = 0; r < 3; ++r) {
                if (k)
                    hipLaunchKernelGGL(rotate_kernel<true>, dim3(blocks), dim3(256), 0, 0, out, sh, iters);
                else
                    hipLaunchKernelGGL(rotate_kernel<false>, dim3(blocks), dim3(256), 0, 0, out, sh, iters);
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms[k], e0, e1));
            ms[k] /= 3;
        }
        const double cyc = 2.4e9 * 1e-3 * prop.multiProcessorCount / insts;  // CU-cycles per wave-instruction per ms
        std::printf("%d %.4f %.4f %.2f %.2f\n", s, ms[0], ms[1], ms[0] * cyc, ms[1] * cyc);
    }
    CK(hipFree(out));
    return 0;
}
