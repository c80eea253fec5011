// graph_branch.hip -- do two branches of a captured HIP graph run concurrently? (development probe)
//   hipcc --offload-arch=gfx950 -O2 -o tools/mb/graph_branch tools/mb/graph_branch.hip && tools/mb/graph_branch
// Branch A: NA one-workgroup kernels that each spin TA us, chained on stream s1; branch B: ONE one-workgroup kernel
// that spins TB us on stream s2, forked from s1 after A's first kernel (or before it). Neither touches memory, so
// concurrent branches take max(A, B) per replay and serialised ones A + B. The learner captures its update with two
// such branches (learner_engine.py _pair).
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void spin(long ticks, int* sink) {   // s_memrealtime: 100 MHz
    const long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
    if (threadIdx.x == 0 && ticks < 0) *sink = 1;
}

static float replay_us(hipGraphExec_t ge, hipStream_t s) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < 20; ++r) {
        CK(hipEventRecord(a, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        best = ms * 1e3f < best ? ms * 1e3f : best;
    }
    return best;
}

int main(int argc, char** argv) {
    const int NA = argc > 1 ? atoi(argv[1]) : 25;
    const long TA = 400, TB = 10000;   // ticks of 10 ns: 4 us and 100 us
    int* sink;
    CK(hipMalloc(&sink, 4));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t fork, join;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    const char* names[] = {"A alone", "B alone", "B forked first", "B forked after A's first kernel", "B captured last"};
    for (int mode = 0; mode < 5; ++mode) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
        CK(hipEventRecord(fork, s1));
        CK(hipStreamWaitEvent(s2, fork, 0));
        const bool a = mode != 1, b = mode != 0;
        if (b && (mode == 1 || mode == 2)) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s2, TB, sink);
        for (int i = 0; i < NA && a; ++i) {
            hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s1, TA, sink);
            if (i == 0 && b && mode == 3) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s2, TB, sink);
        }
        if (b && mode == 4) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s2, TB, sink);
        CK(hipEventRecord(join, s2));
        CK(hipStreamWaitEvent(s1, join, 0));
        CK(hipStreamEndCapture(s1, &g));
        hipGraphExec_t ge;
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s1));
        CK(hipStreamSynchronize(s1));
        printf("NA=%d %-34s %8.1f us per replay\n", NA, names[mode], replay_us(ge, s1));
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}
