// C++-only timing of farms_process_device on a BASELINE config, for the
// hipGraph experiment: without Python the engine binds the HIP
// runtime of /opt/rocm (7.2) rather than the one PyTorch bundles (7.0), whose
// stream capture crashes on the sweeps' launch pattern (tools/graph_capture_probe.hip).
// FARMS_GRAPH=1 captures the sweeps of every call into a graph.
//
// Build: see tools/gpu_graph_ab.sh.  Run: graph_bench [config=3] [steps=5] [filter_size=5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "farms_hip.h"
#include "farms_synth.h"

#define HCHK(x)                                                                  \
    do {                                                                         \
        if ((x) != hipSuccess) { std::fprintf(stderr, "HIP error: %s\n", #x); return 1; } \
    } while (0)

int main(int argc, char **argv) {
    const int config = argc > 1 ? std::atoi(argv[1]) : 3;
    const int steps = argc > 2 ? std::atoi(argv[2]) : 5;
    const int fs = argc > 3 ? std::atoi(argv[3]) : 5;
    farms_synth_params sp;
    if (farms_synth_preset(config, &sp) != 0) return 1;
    const int64_t n = sp.n_events;
    std::vector<int32_t> x(n), y(n), p(n);
    std::vector<uint32_t> t(n);
    if (farms_synth_generate(&sp, x.data(), y.data(), t.data(), p.data()) != n) return 1;
    const uint32_t t0 = t[0];  // vFlow.cpp:194: stamps relative to the first event
    for (auto &v : t) v -= t0;
    for (auto &v : p) v = std::max(v, 0);
    int rv = 0;
    HCHK(hipRuntimeGetVersion(&rv));
    int32_t *dx, *dy, *dp, *ds;
    uint32_t *dt;
    double *dd;
    HCHK(hipMalloc(&dx, 4 * n)); HCHK(hipMalloc(&dy, 4 * n)); HCHK(hipMalloc(&dp, 4 * n));
    HCHK(hipMalloc(&dt, 4 * n)); HCHK(hipMalloc(&ds, 4 * n)); HCHK(hipMalloc(&dd, 6 * 8 * n));
    HCHK(hipMemcpy(dx, x.data(), 4 * n, hipMemcpyHostToDevice));
    HCHK(hipMemcpy(dy, y.data(), 4 * n, hipMemcpyHostToDevice));
    HCHK(hipMemcpy(dt, t.data(), 4 * n, hipMemcpyHostToDevice));
    HCHK(hipMemcpy(dp, p.data(), 4 * n, hipMemcpyHostToDevice));
    farms_records out{};
    out.r_true = dd; out.theta_true = dd + n; out.vx = dd + 2 * n; out.vy = dd + 3 * n;
    out.r_local = dd + 4 * n; out.theta_local = dd + 5 * n; out.scale = ds;
    farms_params prm;
    farms_default_params(&prm);
    prm.width = sp.width; prm.height = sp.height; prm.filter_size = fs; prm.min_inliers = 5;
    farms_handle *h = nullptr;
    if (farms_create(&prm, &h) != FARMS_OK) return 1;
    double best = 1e30, sum = 0.0;
    for (int i = 0; i < steps + 1; ++i) {
        if (farms_reset(h) != FARMS_OK) return 1;
        HCHK(hipDeviceSynchronize());
        const auto a = std::chrono::steady_clock::now();
        if (farms_process_device(h, dx, dy, dt, dp, n, &out) != FARMS_OK) return 1;
        HCHK(hipDeviceSynchronize());
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
        if (i == 0) continue;  // warm-up
        best = std::min(best, ms);
        sum += ms;
    }
    std::vector<int32_t> sc(std::min<int64_t>(n, 1 << 20));
    HCHK(hipMemcpy(sc.data(), ds, 4 * sc.size(), hipMemcpyDeviceToHost));
    long long chk = 0;
    for (int32_t v : sc) chk = chk * 31 + v;
    const char *g = std::getenv("FARMS_GRAPH");
    std::printf("{\"hip_runtime\": %d, \"graph\": %d, \"config\": %d, \"events\": %lld, \"ms_mean\": %.3f, "
                "\"ms_best\": %.3f, \"Mevents_s\": %.3f, \"scale_hash\": %lld}\n",
                rv, g && g[0] == '1', config, (long long)n, sum / steps, best, n / (sum / steps) / 1e3, chk);
    farms_destroy(h);
    return 0;
}
