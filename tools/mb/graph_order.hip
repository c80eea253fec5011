// graph_order.hip -- in which order does the HIP runtime start the branches of a captured graph? (development probe)
//   hipcc --offload-arch=gfx950 -O2 -o tools/mb/graph_order tools/mb/graph_order.hip && tools/mb/graph_order
// Two chains of one-workgroup kernels that each spin a fixed time and record their start (s_memrealtime, 100 MHz):
// chain A (na kernels of ta us) on the capturing stream s1, chain B (nb kernels of tb us) on a second stream s2 forked
// from s1, their first launches captured in the order given. Prints each chain's first and last start relative to
// the earliest start of the replay: whether the second branch waits for the first one's dispatch, and for which one.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void spin(long ticks, unsigned long long* t0, int slot) {
    const long s = __builtin_amdgcn_s_memrealtime();
    t0[slot * 64 + threadIdx.x] = (unsigned long long)s;   // (every lane: a per-lane vector store)
    while (__builtin_amdgcn_s_memrealtime() - s < ticks) __builtin_amdgcn_s_sleep(1);
}

static void run(int na, long ta, int nb, long tb, bool b_first, const char* name) {
    unsigned long long* d;
    CK(hipMalloc(&d, 256 * 64 * 8));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t fork, join;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    hipGraph_t g;
    CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
    CK(hipEventRecord(fork, s1));
    CK(hipStreamWaitEvent(s2, fork, 0));
    // the first launch of each chain in the order asked for, then the rest of A, then the rest of B
    if (b_first) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s2, tb, d, 128);
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s1, ta, d, 0);
    if (!b_first) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s2, tb, d, 128);
    for (int i = 1; i < na; ++i) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s1, ta, d, i);
    for (int i = 1; i < nb; ++i) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s2, tb, d, 128 + i);
    CK(hipEventRecord(join, s2));
    CK(hipStreamWaitEvent(s1, join, 0));
    CK(hipStreamEndCapture(s1, &g));
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    static unsigned long long hh[256 * 64];
    unsigned long long h[256];
    for (int rep = 0; rep < 3; ++rep) {   // the last of three replays
        CK(hipGraphLaunch(ge, s1));
        CK(hipStreamSynchronize(s1));
    }
    CK(hipMemcpy(hh, d, sizeof hh, hipMemcpyDeviceToHost));
    for (int i = 0; i < 256; ++i) h[i] = hh[i * 64];
    unsigned long long t0 = ~0ull;
    for (int i = 0; i < na; ++i) t0 = h[i] < t0 ? h[i] : t0;
    for (int i = 0; i < nb; ++i) t0 = h[128 + i] < t0 ? h[128 + i] : t0;
    printf("%-44s A (%2d x %3ld us): first %7.1f last %7.1f us | B (%2d x %3ld us): first %7.1f last %7.1f us\n", name,
           na, ta / 100, (h[0] - t0) / 100.0, (h[na - 1] - t0) / 100.0, nb, tb / 100, (h[128] - t0) / 100.0,
           (h[128 + nb - 1] - t0) / 100.0);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipFree(d));
}

int main() {
    run(25, 400, 1, 10000, false, "long A, one B, B captured second");
    run(25, 400, 1, 10000, true, "long A, one B, B captured first");
    run(5, 400, 25, 400, false, "short A, long B, B captured second");
    run(5, 400, 25, 400, true, "short A, long B, B captured first");
    run(25, 400, 25, 400, false, "equal chains, B captured second");
    run(25, 400, 25, 400, true, "equal chains, B captured first");
    return 0;
}
