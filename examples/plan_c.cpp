// plan_c.cpp -- the C ABI of libtdmpc_hip.so driven from a plain C++ host, no Python and no torch: the drop-in
// boundary as a non-Python caller (a cgo / JNI / N-API stub) would bind it (include/tdmpc_hip.h).
//
//   examples/plan_c [batch] [calls]      (built by tdmpc_amd.build / __graft_entry__.build())
//
// Humanoid-run shapes (obs 67, A 21, L 100, M 512, N 512, P 256, K 64, H 5, 6 iterations): random TOLD
// parameters in the reference state_dict order -> tdmpc_pack_weights; per-env noise streams of
// tdmpc_noise_floats normals and the choice uniforms; a cold tdmpc_plan and warm-started ones timed with HIP
// events. Prints one line "plan_c: ... plan-steps/s ..." and exits non-zero if an action is not finite, or an
// eval-mode action lies outside [-1, 1].
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../include/tdmpc_hip.h"

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
            return 2;                                                                  \
        }                                                                              \
    } while (0)
#define CT(x)                                                                          \
    do {                                                                               \
        int r_ = (x);                                                                  \
        if (r_) {                                                                      \
            fprintf(stderr, "%s failed: %d %s\n", #x, r_, tdmpc_last_error());         \
            return 3;                                                                  \
        }                                                                              \
    } while (0)

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 32, calls = argc > 2 ? atoi(argv[2]) : 20;
    const int O = 67, A = 21, L = 100, M = 512, E = 256, N = 512, P = 256, K = 64, H = 5, I = 6;
    tdmpc_dims d = {};
    d.modality = 0; d.obs_dim = O; d.action_dim = A; d.latent_dim = L; d.mlp_dim = M; d.enc_dim = E;
    d.num_samples = N; d.num_pi = P; d.num_elites = K; d.max_horizon = H; d.max_iterations = I; d.max_batch = B;
    if (tdmpc_abi_version() != TDMPC_ABI_VERSION) { fprintf(stderr, "ABI mismatch\n"); return 1; }
    tdmpc_sizes sz;
    CT(tdmpc_sizes_for(&d, &sz));

    // TOLD parameters, reference state_dict order (include/tdmpc_hip.h, tdmpc_num_param_tensors)
    std::vector<std::pair<int, int>> shapes = {{E, O}, {E, 1}, {L, E}, {L, 1}};   // _encoder.0 / .2
    auto mlp = [&](int in, int out) {
        shapes.insert(shapes.end(), {{M, in}, {M, 1}, {M, M}, {M, 1}, {out, M}, {out, 1}});
    };
    mlp(L + A, L);   // _dynamics
    mlp(L + A, 1);   // _reward
    mlp(L, A);       // _pi
    for (int q = 0; q < 2; ++q)   // _Q1, _Q2: Linear, LayerNorm, Linear, LayerNorm, Linear
        shapes.insert(shapes.end(), {{M, L + A}, {M, 1}, {M, 1}, {M, 1}, {M, M}, {M, 1}, {M, 1}, {M, 1}, {1, M}, {1, 1}});
    if ((int)shapes.size() != tdmpc_num_param_tensors(&d)) { fprintf(stderr, "tensor count\n"); return 1; }
    std::mt19937 rng(7);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<float*> dev;
    for (auto [r, c] : shapes) {
        std::vector<float> h((size_t)r * c);
        const float s = 1.f / std::sqrt((float)c);
        for (auto& v : h) v = nd(rng) * s;
        float* p;
        CK(hipMalloc(&p, h.size() * 4));
        CK(hipMemcpy(p, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        dev.push_back(p);
    }
    float** tens;
    CK(hipHostMalloc(&tens, dev.size() * sizeof(float*)));   // the pointer array is read on the host
    for (size_t i = 0; i < dev.size(); ++i) tens[i] = dev[i];

    hipStream_t s;
    CK(hipStreamCreate(&s));
    void *packed, *ws;
    CK(hipMalloc(&packed, sz.packed_weight_bytes));
    CK(hipMemset(packed, 0, sz.packed_weight_bytes));   // zero-filled once and announced (tdmpc_hip.h)
    CT(tdmpc_pack_forget(packed));
    CK(hipMalloc(&ws, sz.workspace_bytes));
    CT(tdmpc_pack_weights(&d, tens, (int)dev.size(), packed, sz.packed_weight_bytes, s));

    const size_t nf = tdmpc_noise_floats(&d, H, I);
    std::vector<float> hn(nf * B), ho((size_t)B * O);
    for (auto& v : hn) v = nd(rng);
    for (auto& v : ho) v = nd(rng);
    std::vector<double> hu(B);
    std::uniform_real_distribution<double> ud(0.0, 1.0);
    for (auto& v : hu) v = ud(rng);
    float *noise, *obs, *prev, *act, *met;
    double* u;
    CK(hipMalloc(&noise, hn.size() * 4));
    CK(hipMalloc(&obs, ho.size() * 4));
    CK(hipMalloc(&u, B * 8));
    CK(hipMalloc(&prev, (size_t)B * H * A * 4));
    CK(hipMalloc(&act, (size_t)B * A * 4));
    CK(hipMalloc(&met, (size_t)B * 2 * 4));
    CK(hipMemcpy(noise, hn.data(), hn.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(obs, ho.data(), ho.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(u, hu.data(), B * 8, hipMemcpyHostToDevice));

    tdmpc_plan_params p = {};
    p.horizon = H; p.iterations = I; p.batch = B; p.min_std = 0.05f; p.temperature = 0.5f;
    p.momentum = 0.1f; p.one_minus_momentum = (float)(1.0 - 0.1); p.std_floor = 0.05f; p.path = TDMPC_PATH_AUTO;
    double g = 1.0;
    for (int t = 0; t <= H; ++t) { p.discount_pow[t] = (float)g; g *= 0.99; }
    auto plan = [&]() {
        return tdmpc_plan(&d, &p, packed, obs, 0, noise, u, prev, act, met, nullptr, nullptr, nullptr, nullptr,
                          nullptr, ws, sz.workspace_bytes, s);
    };
    CT(plan());                 // cold start
    p.warm_start = 1;
    CT(plan());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < calls; ++i) CT(plan());
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<float> ha((size_t)B * A);
    CK(hipMemcpy(ha.data(), act, ha.size() * 4, hipMemcpyDeviceToHost));
    // training mode returns mean + std * noise, unclamped as in the reference (tdmpc.py:160-162): finite only;
    // eval mode returns the elite mean of clamped actions: inside [-1, 1]
    int bad = 0;
    for (float v : ha) bad += !std::isfinite(v);
    p.eval_mode = 1;
    CT(plan());
    std::vector<float> he((size_t)B * A);
    CK(hipMemcpy(he.data(), act, he.size() * 4, hipMemcpyDeviceToHost));
    for (float v : he) bad += !(std::isfinite(v) && std::fabs(v) <= 1.f + 1e-6f);
    printf("plan_c: batch %d, %d calls, %.3f ms per call, %.1f plan-steps/s, action[0][0] %.6f, bad %d\n", B, calls,
           ms / calls, B * calls / (ms * 1e-3), ha[0], bad);
    return bad ? 4 : 0;
}
