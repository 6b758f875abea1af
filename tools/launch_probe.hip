// launch_probe.hip -- host cost of the HIP calls a DL-SCL chain enqueues (tools only, not the product):
// hipLaunchKernel of an empty kernel (normal / highest-priority stream, a 368-byte parameter block
// like pscl_decode_params, dynamic LDS), hipMemsetAsync, hipEventRecord, hipStreamWaitEvent, and
// a captured HIP graph of the same launches replayed.
//   hipcc --offload-arch=gfx950 -O2 tools/launch_probe.hip -o /tmp/launch_probe && /tmp/launch_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

struct Big {
    char b[368];
};

__global__ void k_empty(int* p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 1;
}
__global__ void k_big(const Big B) {
    if (B.b[0] == 7 && threadIdx.x == 1000) printf("x");
}
// a long-running kernel occupying every CU (the baseline decode beside the chain)
__global__ void k_spin(long long cycles) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(8);
}
__global__ void k_lds(int* p) {
    extern __shared__ int s[];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = s[5];
}

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e = (x);                                                \
        if (e != hipSuccess) {                                             \
            printf("%s: %s\n", #x, hipGetErrorString(e));                  \
            return 1;                                                      \
        }                                                                  \
    } while (0)

using clk = std::chrono::steady_clock;
static double us_since(clk::time_point a, int n) {
    return std::chrono::duration<double, std::micro>(clk::now() - a).count() / n;
}

int main() {
    int least = 0, greatest = 0;
    CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    hipStream_t s0, s1, s2;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithPriority(&s1, hipStreamNonBlocking, greatest));
    CK(hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, greatest));
    int* d;
    CK(hipMalloc(&d, 1 << 20));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    Big B = {};
    const int n = 2000;
    for (int rep = 0; rep < 2; ++rep) {
        auto a = clk::now();
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_empty, dim3(512), dim3(256), 0, s0, d);
        printf("empty launch, normal stream         %7.2f us\n", us_since(a, n));
        CK(hipStreamSynchronize(s0));
        a = clk::now();
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_empty, dim3(512), dim3(256), 0, s1, d);
        printf("empty launch, high-priority stream  %7.2f us\n", us_since(a, n));
        CK(hipStreamSynchronize(s1));
        a = clk::now();
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_big, dim3(512), dim3(256), 0, s1, B);
        printf("368-byte params, high priority      %7.2f us\n", us_since(a, n));
        CK(hipStreamSynchronize(s1));
        a = clk::now();
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_lds, dim3(512), dim3(256), 16384, s1, d);
        printf("16 KB dynamic LDS, high priority    %7.2f us\n", us_since(a, n));
        CK(hipStreamSynchronize(s1));
        a = clk::now();
        for (int i = 0; i < n; ++i) CK(hipMemsetAsync(d, 0, 64, s1));
        printf("hipMemsetAsync 64 B                 %7.2f us\n", us_since(a, n));
        CK(hipStreamSynchronize(s1));
        a = clk::now();
        for (int i = 0; i < n; ++i) {
            CK(hipEventRecord(ev, s1));
            CK(hipStreamWaitEvent(s2, ev, 0));
        }
        printf("event record + wait (pair)          %7.2f us\n", us_since(a, n));
        CK(hipStreamSynchronize(s1));
        CK(hipStreamSynchronize(s2));
        // cross-stream chain like a retry round: launch s1, record, s2 waits, launch s2, launch s1
        a = clk::now();
        for (int i = 0; i < n / 4; ++i) {
            hipLaunchKernelGGL(k_big, dim3(512), dim3(256), 0, s1, B);
            CK(hipEventRecord(ev, s1));
            CK(hipStreamWaitEvent(s2, ev, 0));
            hipLaunchKernelGGL(k_big, dim3(512), dim3(256), 0, s2, B);
            hipLaunchKernelGGL(k_big, dim3(512), dim3(256), 0, s2, B);
            hipLaunchKernelGGL(k_lds, dim3(512), dim3(256), 16384, s1, d);
        }
        printf("retry-round pattern (4 launches)    %7.2f us per round\n", us_since(a, n / 4));
        CK(hipStreamSynchronize(s1));
        CK(hipStreamSynchronize(s2));
    }
    // the retry-round pattern enqueued while a long kernel occupies the GPU (normal-priority s0)
    for (int pri = 0; pri < 2; ++pri) {
        hipStream_t a1, a2;
        CK(hipStreamCreateWithPriority(&a1, hipStreamNonBlocking, pri ? greatest : least));
        CK(hipStreamCreateWithPriority(&a2, hipStreamNonBlocking, pri ? greatest : least));
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(k_spin, dim3(4096), dim3(256), 0, s0, 20000000LL);
            auto a = clk::now();
            for (int i = 0; i < 8; ++i) {
                hipLaunchKernelGGL(k_big, dim3(512), dim3(256), 0, a1, B);
                CK(hipEventRecord(ev, a1));
                CK(hipStreamWaitEvent(a2, ev, 0));
                hipLaunchKernelGGL(k_big, dim3(512), dim3(256), 0, a2, B);
                hipLaunchKernelGGL(k_big, dim3(512), dim3(256), 0, a2, B);
                hipLaunchKernelGGL(k_lds, dim3(512), dim3(256), 16384, a1, d);
            }
            printf("round pattern under load, %s  %7.2f us per round\n", pri ? "high prio" : "normal   ", us_since(a, 8));
            a = clk::now();
            for (int i = 0; i < 32; ++i) hipLaunchKernelGGL(k_big, dim3(512), dim3(256), 0, a1, B);
            printf("   plain launches under load         %7.2f us\n", us_since(a, 32));
            CK(hipDeviceSynchronize());
        }
        CK(hipStreamDestroy(a1));
        CK(hipStreamDestroy(a2));
    }
    // the same 8 rounds captured as one graph, replayed
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s1, hipStreamCaptureModeRelaxed));
    for (int r = 0; r < 8; ++r) {
        hipLaunchKernelGGL(k_big, dim3(512), dim3(256), 0, s1, B);
        CK(hipEventRecord(ev, s1));
        CK(hipStreamWaitEvent(s2, ev, 0));
        hipLaunchKernelGGL(k_big, dim3(512), dim3(256), 0, s2, B);
        hipLaunchKernelGGL(k_big, dim3(512), dim3(256), 0, s2, B);
        hipLaunchKernelGGL(k_lds, dim3(512), dim3(256), 16384, s1, d);
    }
    hipEvent_t ej;
    CK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
    CK(hipEventRecord(ej, s2));
    CK(hipStreamWaitEvent(s1, ej, 0));
    CK(hipStreamEndCapture(s1, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 2; ++rep) {
        auto a = clk::now();
        for (int i = 0; i < 200; ++i) CK(hipGraphLaunch(ge, s1));
        printf("graph of 8 rounds (32 kernels)      %7.2f us per launch\n", us_since(a, 200));
        auto b = clk::now();
        CK(hipStreamSynchronize(s1));
        printf("   ... GPU drain                    %7.2f us per graph\n", us_since(b, 200));
    }
    printf("done\n");
    return 0;
}
