// Probe of the round-1 hipGraph capture crash ("No hipGraph for
// the sweeps"): captures the engine's three-stream launch pattern with trivial
// kernels and times hipStreamEndCapture + hipGraphInstantiate as the number of
// pooling super-chunks grows, with and without the chain stream's wait on the
// pooling launch two super-chunks back (the ring-reuse edge).
//
// Per super-chunk S (as in farms_fit_device / farms_pool_device):
//   F: `fits` launches, record fit(S)
//   C: wait fit(S) [, wait pool(S-2)], 3 launches (flow, chain, descriptors), record cand(S)
//   P: wait cand(S), `pools` launches, record pool(S)
// The run climbs S and stops once one capture takes longer than the limit, so
// a super-linear cost shows as a growth curve, not as a crash.
//
// Build: hipcc --offload-arch=gfx950 -O2 -o build/graph_capture_probe tools/graph_capture_probe.hip
//        (links the ROCm 7.2 HIP runtime of /opt/rocm), and with -DGRAPH_PROBE_LIB -shared -fPIC as
//        build/libgraph_probe.so, which tools/graph_probe_torch.py loads after `import torch` so that
//        it binds the HIP runtime PyTorch bundles (the one the engine runs on under Python).
// Run:   build/graph_capture_probe [limit_ms]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                              \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

__global__ void k_touch(int *p, int v) { p[threadIdx.x] = v; }

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// returns capture (EndCapture) + instantiate ms; nodes out
static double probe(int n_super, int fits, int pools, bool back_edge, double *t_end, double *t_inst, size_t *nodes) {
    hipStream_t F, C, P;
    CHK(hipStreamCreateWithFlags(&F, hipStreamNonBlocking));
    CHK(hipStreamCreateWithFlags(&C, hipStreamNonBlocking));
    CHK(hipStreamCreateWithFlags(&P, hipStreamNonBlocking));
    int *buf;
    CHK(hipMalloc(&buf, 3 * 64 * sizeof(int)));
    std::vector<hipEvent_t> ef(n_super), ec(n_super), ep(n_super);
    for (int s = 0; s < n_super; ++s) {
        CHK(hipEventCreateWithFlags(&ef[s], hipEventDisableTiming));
        CHK(hipEventCreateWithFlags(&ec[s], hipEventDisableTiming));
        CHK(hipEventCreateWithFlags(&ep[s], hipEventDisableTiming));
    }
    hipEvent_t fork;
    CHK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CHK(hipStreamBeginCapture(F, hipStreamCaptureModeGlobal));
    CHK(hipEventRecord(fork, F));
    CHK(hipStreamWaitEvent(C, fork, 0));
    CHK(hipStreamWaitEvent(P, fork, 0));
    for (int s = 0; s < n_super; ++s) {
        for (int f = 0; f < fits; ++f) hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, F, buf, s);
        CHK(hipEventRecord(ef[s], F));
        CHK(hipStreamWaitEvent(C, ef[s], 0));
        if (back_edge && s >= 2) CHK(hipStreamWaitEvent(C, ep[s - 2], 0));
        for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, C, buf + 64, s);
        CHK(hipEventRecord(ec[s], C));
        CHK(hipStreamWaitEvent(P, ec[s], 0));
        for (int k = 0; k < pools; ++k) hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, P, buf + 128, s);
        CHK(hipEventRecord(ep[s], P));
    }
    CHK(hipStreamWaitEvent(F, ec[n_super - 1], 0));
    CHK(hipStreamWaitEvent(F, ep[n_super - 1], 0));
    hipGraph_t g;
    auto t0 = std::chrono::steady_clock::now();
    CHK(hipStreamEndCapture(F, &g));
    *t_end = ms_since(t0);
    CHK(hipGraphGetNodes(g, nullptr, nodes));
    hipGraphExec_t ge;
    t0 = std::chrono::steady_clock::now();
    CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    *t_inst = ms_since(t0);
    CHK(hipGraphLaunch(ge, F));
    CHK(hipStreamSynchronize(F));
    CHK(hipGraphExecDestroy(ge));
    CHK(hipGraphDestroy(g));
    for (int s = 0; s < n_super; ++s) {
        CHK(hipEventDestroy(ef[s]));
        CHK(hipEventDestroy(ec[s]));
        CHK(hipEventDestroy(ep[s]));
    }
    CHK(hipEventDestroy(fork));
    CHK(hipFree(buf));
    CHK(hipStreamDestroy(F));
    CHK(hipStreamDestroy(C));
    CHK(hipStreamDestroy(P));
    return *t_end + *t_inst;
}

extern "C" int graph_probe_run(double limit) {
    // (fits, pools) per super-chunk: the round-2 engine (8 fit launches, one pooling
    // launch), then per-chunk launches on both streams as in round 1 (16 fit chunks
    // of 65,536 and 64 pooling chunks of 8,192 events per super-chunk): up to ~8k nodes
    const int shapes[3][2] = {{8, 1}, {16, 16}, {16, 64}};
    int rv = 0;
    CHK(hipRuntimeGetVersion(&rv));
    std::printf("# HIP runtime %d\n", rv);
    std::printf("fits pools back_edge n_super nodes end_capture_ms instantiate_ms\n");
    for (const auto &sh : shapes) {
        for (int be = 0; be <= 1; ++be) {
            for (int n = 2; n <= 96; n += (n < 16 ? 2 : 16)) {
                double te, ti;
                size_t nodes = 0;
                const double t = probe(n, sh[0], sh[1], be != 0, &te, &ti, &nodes);
                std::printf("%d %d %d %d %zu %.3f %.3f\n", sh[0], sh[1], be, n, nodes, te, ti);
                std::fflush(stdout);
                if (t > limit) {
                    std::printf("# stop: %d super-chunks took %.0f ms (limit %.0f)\n", n, t, limit);
                    break;
                }
            }
        }
    }
    return 0;
}

#ifndef GRAPH_PROBE_LIB
int main(int argc, char **argv) { return graph_probe_run(argc > 1 ? std::atof(argv[1]) : 3000.0); }
#endif
