// Host-side enqueue costs of the HIP runtime (diagnostic for the host path):
// per-call host time of kernel launches (small and 400-B arguments),
// hipEventRecord, cross-stream hipStreamWaitEvent and hipMemcpyAsync D2H into
// pinned memory, on non-blocking streams as the engine uses them.
// Build: hipcc --offload-arch=gfx950 -O2 -shared -fPIC tools/launch_probe.hip -o tools/build/liblaunch_probe.so
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

struct Big { long long v[50]; };
__global__ void k_small(int *p) { if (p && threadIdx.x == 1000) p[0] = 1; }
__global__ void k_big(Big b) { if (b.v[0] == 12345 && threadIdx.x == 1000) ((int *)b.v[1])[0] = 1; }
// device -> host stores (grid-stride, 16-B moves)
__global__ void k_store(const double2 *src, double2 *dst, long long n2) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n2; i += (long long)gridDim.x * blockDim.x)
        dst[i] = src[i];
}
// one wave that spins for `ticks` of the 100 MHz real-time counter (ends on its own)
__global__ void k_spin(long long ticks, int *p) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    if (p && threadIdx.x == 1000) p[0] = 1;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x) do { if ((x) != hipSuccess) { std::printf("fail %s\n", #x); return 1; } } while (0)

extern "C" int launch_probe(int iters) {
    hipStream_t s[4];
    for (int i = 0; i < 4; ++i) CK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
    hipEvent_t ev[4096];
    for (int i = 0; i < 4096; ++i) CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    int *d;
    CK(hipMalloc(&d, 64 << 20));
    void *hp;
    CK(hipHostMalloc(&hp, 64 << 20, hipHostMallocDefault));
    Big b{};
    auto run = [&](const char *what, auto fn) -> int {
        for (int i = 0; i < 50; ++i) fn(i);
        if (hipDeviceSynchronize() != hipSuccess) return 1;
        const double t0 = now_us();
        for (int i = 0; i < iters; ++i) fn(i);
        const double t1 = now_us();
        if (hipDeviceSynchronize() != hipSuccess) return 1;
        const double t2 = now_us();
        std::printf("%-44s enqueue %8.2f us/call   drain %8.2f us/call\n", what, (t1 - t0) / iters, (t2 - t0) / iters);
        return 0;
    };
    int rc = 0;
    rc |= run("launch, 8-B arg", [&](int) { hipLaunchKernelGGL(k_small, dim3(1024), dim3(64), 0, s[0], d); });
    rc |= run("launch, 400-B arg", [&](int) { hipLaunchKernelGGL(k_big, dim3(1024), dim3(64), 0, s[0], b); });
    rc |= run("launch + hipEventRecord", [&](int i) {
        hipLaunchKernelGGL(k_big, dim3(1024), dim3(64), 0, s[0], b);
        (void)hipEventRecord(ev[i % 4096], s[0]);
    });
    rc |= run("launch on s1 + wait(event of s0) + record", [&](int i) {
        hipLaunchKernelGGL(k_big, dim3(1024), dim3(64), 0, s[0], b);
        (void)hipEventRecord(ev[i % 4096], s[0]);
        (void)hipStreamWaitEvent(s[1], ev[i % 4096], 0);
        hipLaunchKernelGGL(k_big, dim3(1024), dim3(64), 0, s[1], b);
    });
    rc |= run("3 streams: F launch+rec, C wait+launch, P wait", [&](int i) {
        hipLaunchKernelGGL(k_big, dim3(1024), dim3(64), 0, s[0], b);
        (void)hipEventRecord(ev[(2 * i) % 4096], s[0]);
        (void)hipStreamWaitEvent(s[1], ev[(2 * i) % 4096], 0);
        hipLaunchKernelGGL(k_big, dim3(1024), dim3(64), 0, s[1], b);
        (void)hipEventRecord(ev[(2 * i + 1) % 4096], s[1]);
        (void)hipStreamWaitEvent(s[2], ev[(2 * i + 1) % 4096], 0);
        hipLaunchKernelGGL(k_big, dim3(1024), dim3(64), 0, s[2], b);
    });
    rc |= run("D2H 1 MB into pinned (s3)", [&](int i) {
        (void)hipMemcpyAsync((char *)hp + (size_t)(i % 32) * (1 << 20), (char *)d + (size_t)(i % 32) * (1 << 20),
                             1 << 20, hipMemcpyDeviceToHost, s[3]);
    });
    rc |= run("H2D 1 MB from pinned (s3)", [&](int i) {
        (void)hipMemcpyAsync((char *)d + (size_t)(i % 32) * (1 << 20), (char *)hp + (size_t)(i % 32) * (1 << 20),
                             1 << 20, hipMemcpyHostToDevice, s[3]);
    });
    // long kernels (50 us each): is the host enqueue paced by the GPU?
    const long long T = 5000;
    rc |= run("spin50 + record (F)", [&](int i) {
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s[0], T, d);
        (void)hipEventRecord(ev[i % 4096], s[0]);
    });
    rc |= run("spin50 F + rec, C waits + spin50", [&](int i) {
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s[0], T, d);
        (void)hipEventRecord(ev[i % 4096], s[0]);
        (void)hipStreamWaitEvent(s[1], ev[i % 4096], 0);
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s[1], T, d);
    });
    rc |= run("spin50 F only, 4 launches", [&](int) {
        for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s[0], T, d);
    });
    // kernel stores into pinned host memory: GB/s by grid size (64 MB per launch)
    for (int wgs : {32, 128, 512, 2048}) {
        char name[64];
        std::snprintf(name, sizeof(name), "k_store 64 MB -> pinned, %d WGs", wgs);
        const int it = 20;
        const double t0 = now_us();
        for (int i = 0; i < it; ++i)
            hipLaunchKernelGGL(k_store, dim3(wgs), dim3(256), 0, s[3], (const double2 *)d, (double2 *)hp, (64ll << 20) / 16);
        if (hipStreamSynchronize(s[3]) != hipSuccess) return 1;
        const double t1 = now_us();
        std::printf("%-44s %8.1f GB/s\n", name, it * 64.0 * (1 << 20) / ((t1 - t0) * 1e3));
    }
    {
        const int it = 20;
        const double t0 = now_us();
        for (int i = 0; i < it; ++i) (void)hipMemcpyAsync(hp, d, 64 << 20, hipMemcpyDeviceToHost, s[3]);
        if (hipStreamSynchronize(s[3]) != hipSuccess) return 1;
        const double t1 = now_us();
        std::printf("%-44s %8.1f GB/s\n", "hipMemcpyAsync 64 MB D2H", it * 64.0 * (1 << 20) / ((t1 - t0) * 1e3));
    }
    for (int i = 0; i < 4; ++i) (void)hipStreamDestroy(s[i]);
    for (int i = 0; i < 4096; ++i) (void)hipEventDestroy(ev[i]);
    (void)hipFree(d);
    (void)hipHostFree(hp);
    return rc;
}
