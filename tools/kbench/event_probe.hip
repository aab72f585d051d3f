// Cost of an event record between back-to-back kernels on one stream (the decoder records its
// workspace event after every call).  Per mode, K launches of a short kernel,
// timed by one event pair around them; per-launch time in microseconds:
//   plain        kernel only
//   rec_default  + hipEventRecord(default event)
//   rec_notiming + hipEventRecord(hipEventDisableTiming)
//   rec_nofence  + hipEventRecord(hipEventDisableTiming | hipEventDisableSystemFence)
//   rec_timing_nofence + hipEventRecord(hipEventDisableSystemFence)
//   ext_default  hipExtLaunchKernelGGL with the default event as its stop event
//   ext_notiming / ext_nofence   the same with the other events
// then a second stream waits on each ext-recorded event and launches a kernel that checks the first
// stream's last write (ordering through an event attached to a kernel).
//   hipcc --offload-arch=gfx950 -O3 tools/kbench/event_probe.hip -o tools/kbench/event_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__global__ void work(float* x, int iters, int tag)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float v = x[i];
    for (int k = 0; k < iters; ++k) v = v * 0.999f + 0.001f;
    x[i] = v;
    if (i == 0) reinterpret_cast<int*>(x)[-1] = tag;
}

__global__ void check(const float* x, int want, int* out)
{
    if (threadIdx.x == 0) *out = reinterpret_cast<const int*>(x)[-1] == want;
}

int main(int argc, char** argv)
{
    const int K = argc > 1 ? std::atoi(argv[1]) : 2000;
    const int blocks = 1024, threads = 256, iters = argc > 2 ? std::atoi(argv[2]) : 64;
    float* buf;
    CK(hipMalloc(&buf, (blocks * threads + 64) * sizeof(float)));
    CK(hipMemset(buf, 0, (blocks * threads + 64) * sizeof(float)));
    float* x = buf + 64;
    int* flag;
    CK(hipMalloc(&flag, sizeof(int)));
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t t0, t1, evd, evn, evf, evtf;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    CK(hipEventCreate(&evd));
    CK(hipEventCreateWithFlags(&evn, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&evf, hipEventDisableTiming | hipEventDisableSystemFence));
    CK(hipEventCreateWithFlags(&evtf, hipEventDisableSystemFence));
    struct Mode { const char* name; int kind; hipEvent_t ev; };
    const Mode modes[] = {{"plain", 0, nullptr},          {"rec_default", 1, evd},  {"rec_notiming", 1, evn},
                          {"rec_nofence", 1, evf},        {"rec_timing_nofence", 1, evtf},
                          {"ext_default", 2, evd},        {"ext_notiming", 2, evn}, {"ext_nofence", 2, evf},
                          {"ext_timing_nofence", 2, evtf}};
    for (int rep = 0; rep < 3; ++rep) {
        for (const Mode& m : modes) {
            for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(work, dim3(blocks), dim3(threads), 0, s, x, iters, w);
            CK(hipStreamSynchronize(s));
            CK(hipEventRecord(t0, s));
            for (int k = 0; k < K; ++k) {
                if (m.kind == 2) {
                    hipExtLaunchKernelGGL(work, dim3(blocks), dim3(threads), 0, s, nullptr, m.ev, 0, x, iters, k);
                } else {
                    hipLaunchKernelGGL(work, dim3(blocks), dim3(threads), 0, s, x, iters, k);
                    if (m.kind == 1) CK(hipEventRecord(m.ev, s));
                }
            }
            CK(hipGetLastError());
            CK(hipEventRecord(t1, s));
            int ok = -1;
            if (m.ev) {  // ordering through the event: the second stream sees the last kernel's write
                CK(hipStreamWaitEvent(s2, m.ev, 0));
                hipLaunchKernelGGL(check, dim3(1), dim3(64), 0, s2, x, K - 1, flag);
                CK(hipStreamSynchronize(s2));
                CK(hipMemcpy(&ok, flag, sizeof(int), hipMemcpyDeviceToHost));
            }
            CK(hipEventSynchronize(t1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, t0, t1));
            std::printf("rep %d %-20s %8.3f us per launch  ordered=%d\n", rep, m.name, 1e3 * ms / K, ok);
        }
    }
    return 0;
}
