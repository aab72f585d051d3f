// ds_permute_b32 when several lanes push to one lane: which source wins, and what a lane no one
// pushes to receives.  Prints, per destination lane, the source lane whose value arrived.
//   hipcc --offload-arch=gfx950 -O3 -o tools/kbench/permute_collide tools/kbench/permute_collide.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void collide(int* out, int mode)
{
    const int lane = threadIdx.x & 63;
    int dest;
    if (mode == 0) dest = lane & 31;                 // lanes j and j + 32 -> j
    else if (mode == 1) dest = lane < 61 ? (lane + 7) % 61 : (lane - 61 + 7);  // idle 61..63 collide with 7..9's targets
    else dest = lane < 3 ? lane + 20 : lane;         // low lanes 0..2 collide on 20..22 with the lanes themselves
    out[mode * 64 + lane] = __builtin_amdgcn_ds_permute(dest * 4, lane + 1000);
}

int main()
{
    int* d = nullptr;
    if (hipMalloc(&d, 3 * 64 * sizeof(int)) != hipSuccess) return 1;
    for (int m = 0; m < 3; ++m) hipLaunchKernelGGL(collide, dim3(1), dim3(64), 0, 0, d, m);
    int h[3 * 64];
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    for (int m = 0; m < 3; ++m) {
        std::printf("mode %d:", m);
        for (int l = 0; l < 64; ++l) std::printf(" %d", h[m * 64 + l] >= 1000 ? h[m * 64 + l] - 1000 : -1 - h[m * 64 + l]);
        std::printf("\n");
    }
    hipFree(d);
    return 0;
}
