// Microbenchmark of the planner's kernels in isolation (development tool, not shipped).
// Includes the library source so the internal launchers can be driven directly.
#include "../../tdmpc_amd/csrc/tdmpc_kernels.hip"

#include <vector>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static float time_it(hipStream_t s, int iters, const std::function<void()>& fn) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) fn();
    CK(hipEventRecord(a, s));
    for (int i = 0; i < iters; ++i) fn();
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / iters;
}

int main(int argc, char** argv) {
    int B = argc > 1 ? atoi(argv[1]) : 1;
    tdmpc_dims d{};
    d.modality = 0; d.obs_dim = 67; d.action_dim = 21; d.latent_dim = 100; d.mlp_dim = 512; d.enc_dim = 256;
    d.num_samples = 512; d.num_pi = 256; d.num_elites = 64; d.max_horizon = 5; d.max_iterations = 6; d.max_batch = B;
    tdmpc_sizes sz;
    if (tdmpc_sizes_for(&d, &sz)) { printf("sizes failed\n"); return 1; }
    void *packed, *ws; float* noise; double* u; float *prev, *act, *met, *obs;
    CK(hipMalloc(&packed, sz.packed_weight_bytes)); CK(hipMalloc(&ws, sz.workspace_bytes));
    CK(hipMalloc(&noise, sz.noise_floats_per_env * 4 * B)); CK(hipMalloc(&u, 8 * B));
    CK(hipMalloc(&prev, 4 * 5 * 21 * B)); CK(hipMalloc(&act, 4 * 21 * B)); CK(hipMalloc(&met, 8 * B));
    CK(hipMalloc(&obs, 4 * 67 * B));
    // random packed weights / workspace / noise (values ~ N(0, 1/sqrt(512)))
    {
        std::mt19937 g(0); std::normal_distribution<float> nd(0.f, 0.04f);
        std::vector<float> hw(sz.packed_weight_bytes / 4);
        for (auto& x : hw) x = nd(g);
        CK(hipMemcpy(packed, hw.data(), sz.packed_weight_bytes, hipMemcpyHostToDevice));
        std::vector<float> hn(sz.noise_floats_per_env * B);
        std::normal_distribution<float> n1(0.f, 1.f);
        for (auto& x : hn) x = n1(g);
        CK(hipMemcpy(noise, hn.data(), hn.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemset(ws, 0, sz.workspace_bytes));
        std::vector<float> ho(67 * B); for (auto& x : ho) x = n1(g);
        CK(hipMemcpy(obs, ho.data(), ho.size() * 4, hipMemcpyHostToDevice));
        std::vector<double> hu(B, 0.5); CK(hipMemcpy(u, hu.data(), 8 * B, hipMemcpyHostToDevice));
        CK(hipMemset(prev, 0, 4 * 5 * 21 * B));
    }
    hipStream_t s; CK(hipStreamCreate(&s));
    // "s2loop [n]": only the rollout S2 launch (h2 of dynamics+reward, the dominant kernel), n times -- for
    // rocprofv3 --pmc passes whose counters must not mix with other kernels of the same grid size.
    const bool s2loop = argc > 2 && !strcmp(argv[2], "s2loop");
    const int s2n = argc > 3 ? atoi(argv[3]) : 50;
    tdmpc_plan_params p{};
    p.horizon = 5; p.iterations = 6; p.batch = B; p.warm_start = 0; p.eval_mode = 0;
    p.min_std = 0.05f; p.temperature = 0.5f; p.momentum = 0.1f; p.one_minus_momentum = 0.9f; p.std_floor = 0.05f;
    float dd = 1.f; for (int t = 0; t <= 5; ++t) { p.discount_pow[t] = dd; dd *= 0.99f; }
    if (s2loop) {
        Ctx c;
        if (setup_ctx(c, &d, packed, ws, sz.workspace_bytes, B, 5, 6, s)) { printf("ctx failed\n"); return 1; }
        const Layout& w = c.w; const int M = c.M;
        LinArgs a = args0();
        a.M = B * c.N; a.K = M;
        LinProb& p0 = a.p[0];
        p0.A = hop(c.k.H1, c, 0); p0.W = wop(c, w.w2d, M); p0.bias = c.pw + w.b2d;
        p0.C = hout(c.k.H2, c, 0); p0.N = p0.nvalid = p0.nstore = M; p0.epi = EPI_ELU;
        LinProb& p1 = a.p[1];
        p1.A = hop(c.k.H1, c, M / 4); p1.W = wop(c, w.w2r, M); p1.bias = c.pw + w.b2r;
        p1.N = p1.nvalid = M; p1.nstore = 0; p1.epi = EPI_ELU_DOT;
        p1.dotw = c.pw + w.w3r; p1.dot_out = c.k.rpart; p1.dot_ld = M / pick_cfg(a.M, M, M, 0).bw;
        for (int i = 0; i < s2n; ++i)
            if (launch_lin(a, 2, M, 0, PRO_PLAIN, s)) { printf("launch failed %s\n", tdmpc_last_error()); return 1; }
        CK(hipStreamSynchronize(s));
        printf("s2loop B=%d rows=%d launches=%d\n", B, a.M, s2n);
        return 0;
    }
    if (argc > 2 && !strcmp(argv[2], "chainloop")) {
        // only the chain rollout step over the B*N candidate rows, n times (PMC passes)
        Ctx c;
        if (setup_ctx(c, &d, packed, ws, sz.workspace_bytes, B, 5, 6, s)) { printf("ctx failed\n"); return 1; }
        c.path = 2;
        const RowMap rmc = {c.N, c.T, 0};
        for (int i = 0; i < s2n; ++i)
            if (step_next(c, 1, B * c.N, rmc, 0.99f, 0, 0)) { printf("launch failed %s\n", tdmpc_last_error()); return 1; }
        CK(hipStreamSynchronize(s));
        printf("chainloop B=%d rows=%d launches=%d\n", B, B * c.N, s2n);
        return 0;
    }
    if (argc > 2 && !strcmp(argv[2], "sweep")) {
        // tile-shape sweep over the planner's GEMM shapes (rows x N x K x problems), plain ELU epilogue
        Ctx c;
        if (setup_ctx(c, &d, packed, ws, sz.workspace_bytes, B, 5, 6, s)) { printf("ctx failed\n"); return 1; }
        init_attrs();
#define ATTR1(...) CK(hipFuncSetAttribute((const void*)linear_lds_kernel<__VA_ARGS__>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
#define ATTR(...) ATTR1(__VA_ARGS__, true) ATTR1(__VA_ARGS__, false)
        ATTR(1, 1, 2, 2, 32) ATTR(1, 2, 2, 2, 32) ATTR(1, 1, 2, 4, 32) ATTR(1, 2, 2, 4, 32)
#undef ATTR
        const Layout& w = c.w; const int M = c.M;
        struct Shape { const char* name; int rows, n, k, nprob; size_t woff; };
        std::vector<Shape> shapes = {
            {"pi-rows L2 (B*P x 512 x 512)", B * c.P, M, M, 1, w.w2d},
            {"S2 rollout (B*N x 512 x 512 x2)", B * c.N, M, M, 2, w.w2d},
            {"S2 all rows (B*T x 512 x 512 x2)", B * c.T, M, M, 2, w.w2d},
            {"pi2 all rows (B*T x 512 x 512)", B * c.T, M, M, 1, w.w2d},
            {"S1 rollout (B*N x 1024 x Kx)", B * c.N, 2 * M, c.Kx, 1, w.w1x},
            {"S1 all rows (B*T x 1024 x Kx)", B * c.T, 2 * M, c.Kx, 1, w.w1x},
            {"S3 rollout (B*N x 100 x 512)", B * c.N, w.L, M, 1, w.w3d},
        };
        for (auto& sh : shapes) {
            LinArgs a = args0();
            a.M = sh.rows; a.K = sh.k;
            for (int q = 0; q < sh.nprob; ++q) {
                LinProb& p = a.p[q];
                p.A = hop(c.k.H1, c, 0); p.W = wop(c, sh.woff, sh.k); p.bias = c.pw + w.b2d;
                p.C = hout(c.k.H2, c, q * (sh.n / 4)); p.N = p.nvalid = p.nstore = sh.n; p.epi = EPI_ELU;
            }
            printf("%s\n", sh.name);
            auto run = [&](const char* nm, const std::function<int()>& f) {
                float us = time_it(s, 200, [&] { if (f()) { printf("launch failed\n"); exit(1); } });
                const double fl = 2.0 * sh.rows * sh.n * sh.k * sh.nprob;
                printf("   %-26s %8.2f us  %6.1f TF\n", nm, us, fl / us * 1e-6);
            };
            const int np = sh.nprob, nm = sh.n;
            run("auto (launch_lin)", [&] { return launch_lin(a, np, nm, 0, PRO_PLAIN, s); });
            if (sh.k >= 64) {
                run("lds 128x128 8w", [&] { return launch_lds_t<2, 1, 2, 4, 32>(a, np, nm, s); });
                run("lds 192x128 8w", [&] { return launch_lds_t<3, 1, 2, 4, 32>(a, np, nm, s); });
                run("lds 128x64 4w", [&] { return launch_lds_t<2, 1, 2, 2, 32>(a, np, nm, s); });
                run("lds 64x64 4w", [&] { return launch_lds_t<1, 1, 2, 2, 32>(a, np, nm, s); });
                run("lds 64x128 4w", [&] { return launch_lds_t<1, 2, 2, 2, 32>(a, np, nm, s); });
                run("lds 64x128 8w", [&] { return launch_lds_t<1, 1, 2, 4, 32>(a, np, nm, s); });
                if (nm % 256 == 0) run("lds 64x256 8w", [&] { return launch_lds_t<1, 2, 2, 4, 32>(a, np, nm, s); });
            }
            if (sh.k <= 1024) {
                const int kch = sh.k > 256 ? 64 : 32;
                if (kch == 64) {
                    run("lat 32x32 ksplit", [&] { return launch_lin_t<1, 1, 1, 1, 0, 64, false>(a, np, nm, 1, s); });
                    run("lat 32x64 ksplit", [&] { return launch_lin_t<1, 2, 1, 1, 0, 64, false>(a, np, nm, 2, s); });
                } else {
                    run("lat 32x32 ksplit", [&] { return launch_lin_t<1, 1, 1, 1, 0, 32, false>(a, np, nm, 1, s); });
                    run("lat 32x64 ksplit", [&] { return launch_lin_t<1, 2, 1, 1, 0, 32, false>(a, np, nm, 2, s); });
                }
            }
        }
        CK(hipStreamSynchronize(s));
        return 0;
    }
    for (int path = 0; path <= 2; ++path) {
        p.path = path;
        float t_plan = time_it(s, 20, [&] {
            int rc = tdmpc_plan(&d, &p, packed, obs, 0, noise, u, prev, act, met, nullptr, nullptr, nullptr, nullptr,
                                nullptr, ws, sz.workspace_bytes, s);
            if (rc) { printf("plan rc %d %s\n", rc, tdmpc_last_error()); exit(1); }
        });
        printf("B=%d full plan (path %d): %.1f us\n", B, path, t_plan);
    }
    p.path = 0;
    Ctx c;
    setup_ctx(c, &d, packed, ws, sz.workspace_bytes, B, 5, 6, s);
    const RowMap rm = {c.N, c.T, 0};
    const RowMap all = {c.T, c.T, 0};
    struct Case { const char* name; std::function<void()> fn; };
    std::vector<Case> cases;
    // one rollout step / terminal heads on each path
    for (int path = 1; path <= 2; ++path) {
        const char* pn = path == 1 ? "layered" : "chain";
        static char nm[8][64];
        snprintf(nm[path * 3 - 3], 64, "step_next N rows (%s)", pn);
        snprintf(nm[path * 3 - 2], 64, "policy T rows (%s)", pn);
        snprintf(nm[path * 3 - 1], 64, "terminal_q T rows (%s)", pn);
        cases.push_back({nm[path * 3 - 3], [&, path] { c.path = path; step_next(c, 1, B * c.N, rm, 0.99f, 0, 0); }});
        cases.push_back({nm[path * 3 - 2], [&, path] { c.path = path; policy(c, 5, B * c.T, all, noise, c.eps_env, c.T, 0, 0.05f); }});
        cases.push_back({nm[path * 3 - 1], [&, path] { c.path = path; terminal_q(c, 0.95f); }});
    }
    cases.push_back({"step_next T rows (chain)", [&] { c.path = 2; step_next(c, 1, B * c.T, all, 0.99f, 0, 0); }});
    cases.push_back({"policy P rows (chain)", [&] { c.path = 2; policy(c, 1, B * c.P, RowMap{c.P, c.T, c.N}, noise, c.eps_env, c.P, 0, 0.05f); }});
    cases.push_back({"policy P rows (layered)", [&] { c.path = 1; policy(c, 1, B * c.P, RowMap{c.P, c.T, c.N}, noise, c.eps_env, c.P, 0, 0.05f); }});
    cases.push_back({"encode", [&] { encode(c, obs, 0, B, prev, 0); }});
    for (auto& cs : cases) printf("%-32s %8.2f us\n", cs.name, time_it(s, 200, cs.fn));
    c.path = 0;
    if (argc > 2 && !strcmp(argv[2], "chain")) return 0;
    // per-layer: S2 only
    {
        const Layout& w = c.w; const int M = c.M;
        LinArgs a = args0();
        a.M = B * c.N; a.K = M;
        LinProb& p0 = a.p[0];
        p0.A = hop(c.k.H1, c, 0); p0.W = wop(c, w.w2d, M); p0.bias = c.pw + w.b2d;
        p0.C = hout(c.k.H2, c, 0); p0.N = p0.nvalid = p0.nstore = M; p0.epi = EPI_ELU;
        LinProb& p1 = a.p[1];
        p1.A = hop(c.k.H1, c, M / 4); p1.W = wop(c, w.w2r, M); p1.bias = c.pw + w.b2r;
        p1.N = p1.nvalid = M; p1.nstore = 0; p1.epi = EPI_ELU_DOT;
        p1.dotw = c.pw + w.w3r; p1.dot_out = c.k.rpart; p1.dot_ld = M / pick_cfg(a.M, M, M, 0).bw;
        printf("%-32s %8.2f us\n", "S2 (WN=1)", time_it(s, 500, [&] { launch_lin(a, 2, M, 0, PRO_PLAIN, s); }));
        p1.epi = EPI_ELU; p1.C = hout(c.k.H2, c, M / 4); p1.nstore = M;
        printf("%-32s %8.2f us\n", "S2 (WN=2)", time_it(s, 500, [&] { launch_lin(a, 2, M, 2, PRO_PLAIN, s); }));
        a.p[0].N = 32;
        printf("%-32s %8.2f us\n", "1 col tile x 2 (WN=1)", time_it(s, 500, [&] { launch_lin(a, 2, 32, 1, PRO_PLAIN, s); }));
    }
#ifdef TDMPC_STAMPS
    {
        unsigned long long* dbuf; CK(hipMalloc(&dbuf, 8 * 8 * 8192));
        unsigned int cap = 8192;
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_cap), &cap, 4));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &dbuf, sizeof(dbuf)));
        auto run_case = [&](const char* name, const std::function<void()>& fn, int ysel = -1) {
            for (int i = 0; i < 5; ++i) fn();
            CK(hipStreamSynchronize(s));
            unsigned int zero = 0;
            CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_n), &zero, 4));
            fn();
            CK(hipStreamSynchronize(s));
            unsigned int n; CK(hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_stamp_n), 4));
            n = std::min(n, 8192u);
            std::vector<unsigned long long> h(8 * n);
            CK(hipMemcpy(h.data(), dbuf, 8 * 8 * n, hipMemcpyDeviceToHost));
            if (ysel >= 0) {   // keep the workgroups with blockIdx.y == ysel
                unsigned m = 0;
                for (unsigned i = 0; i < n; ++i)
                    if ((int)((h[8 * i + 6] >> 16) & 0xffff) == ysel) { for (int k = 0; k < 8; ++k) h[8 * m + k] = h[8 * i + k]; ++m; }
                n = m;
            }
            unsigned long long rtmin = ~0ull, rtmax = 0;
            double ph[4] = {0, 0, 0, 0}, phmax[4] = {0, 0, 0, 0};
            int xcc_hist[8] = {0};
            for (unsigned i = 0; i < n; ++i) {
                unsigned long long* o = &h[8 * i];
                rtmin = std::min(rtmin, o[0]); rtmax = std::max(rtmax, o[0]);
                for (int k = 0; k < 4; ++k) { double d = double(o[2 + k] - o[1 + k]); ph[k] += d; phmax[k] = std::max(phmax[k], d); }
                xcc_hist[o[7] & 7]++;
            }
            double span_rt = 0, span_cy = 0;
            unsigned long long rtend = 0;
            for (unsigned i = 0; i < n; ++i) {
                span_rt += double(h[8 * i + 7] >> 8); span_cy += double(h[8 * i + 5] - h[8 * i + 1]);
                rtend = std::max(rtend, h[8 * i] + (h[8 * i + 7] >> 8));
            }
            printf("%s: kernel wall (first start -> last end) %.2f us\n", name, (rtend - rtmin) / 100.0);
            printf("%s: %u WGs, start skew %.2f us, WG span %.2f us @ %.2f GHz, avg cycles: ph0 %.0f ph1 %.0f ph2 %.0f ph3 %.0f | max %.0f %.0f %.0f %.0f | xcc",
                   name, n, (rtmax - rtmin) / 100.0, span_rt / n / 100.0, span_cy / (span_rt * 10.0) , ph[0] / n, ph[1] / n, ph[2] / n, ph[3] / n, phmax[0], phmax[1], phmax[2], phmax[3]);
            for (int k = 0; k < 8; ++k) printf(" %d", xcc_hist[k]);
            printf("\n");
            // xcc of first 16 WGs (blockIdx order)
            std::vector<std::pair<unsigned long long, unsigned long long>> v;
            for (unsigned i = 0; i < n; ++i) v.push_back({h[8 * i + 6], h[8 * i + 7] & 0xff});
            std::sort(v.begin(), v.end());
            printf("   blockIdx->xcc:");
            for (unsigned i = 0; i < std::min(n, 20u); ++i) printf(" %llu:%llu", v[i].first & 0xffff, v[i].second);
            printf("\n");
        };
        const Layout& w = c.w; const int M = c.M;
        LinArgs a = args0();
        a.M = B * c.N; a.K = M;
        LinProb& p0 = a.p[0];
        p0.A = hop(c.k.H1, c, 0); p0.W = wop(c, w.w2d, M); p0.bias = c.pw + w.b2d;
        p0.C = hout(c.k.H2, c, 0); p0.N = p0.nvalid = p0.nstore = M; p0.epi = EPI_ELU;
        a.p[1] = p0;
        a.p[1].A = hop(c.k.H1, c, M / 4); a.p[1].W = wop(c, w.w2r, M); a.p[1].C = hout(c.k.H2, c, M / 4);
        run_case("S2 auto", [&] { launch_lin(a, 2, M, 0, PRO_PLAIN, s); });
        run_case("S2 lds 128x128", [&] { launch_lds_t<2, 1, 2, 4, 32>(a, 2, M, s); });
        run_case("S2 lds 128x128 again", [&] { launch_lds_t<2, 1, 2, 4, 32>(a, 2, M, s); });
        run_case("S2 lds 64x64", [&] { launch_lds_t<1, 1, 2, 2, 32>(a, 2, M, s); });
        LinArgs b = a; b.K = 128; b.p[0].W = wop(c, w.w2d, 128);  b.p[1].W = wop(c, w.w2r, 128);
        run_case("S2 lds 128x128 K=128", [&] { launch_lds_t<2, 1, 2, 4, 32>(b, 2, M, s); });
        LinArgs e = a; e.M = B * c.T;
        run_case("S2 all rows lds 192x128", [&] { launch_lds_t<3, 1, 2, 4, 32>(e, 2, M, s); });
        const RowMap rmc = {c.N, c.T, 0};
        const RowMap allc = {c.T, c.T, 0};
        c.path = 2;
        run_case("chain step dyn (N rows)", [&] { step_next(c, 1, B * c.N, rmc, 0.99f, 0, 0); }, 0);
        run_case("chain step rew (N rows)", [&] { step_next(c, 1, B * c.N, rmc, 0.99f, 0, 0); }, 1);
        run_case("chain pi (T rows)", [&] { policy(c, 5, B * c.T, allc, noise, c.eps_env, c.T, 0, 0.05f); });
        run_case("chain Q (T rows)", [&] { terminal_q(c, 0.95f); }, 0);
        c.path = 0;
    }
#endif
    CK(hipStreamSynchronize(s));
    return 0;
}
