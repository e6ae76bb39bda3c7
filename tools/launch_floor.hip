// launch_floor.hip -- the HIP runtime's own host cost per kernel launch on this box (diagnostics for
// tools/host_probe.py: what part of rsd_svao_frame's host time is librsd and what part is the
// runtime).  Empty kernels with a 64-byte and a 2048-byte argument struct (SvaoArgs is ~2 KB),
// launched back to back on one non-blocking stream, plus hipEventRecord; the GPU queue is drained
// between batches so the host never blocks on a full queue.
// build + run on the GPU box: hipcc --offload-arch=gfx950 -O2 tools/launch_floor.hip -o /tmp/lf && /tmp/lf
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>

struct Small {
    float v[16];
};
struct Big {
    float v[512];
};

__global__ void k_small(Small s, float* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && s.v[0] < -1.0f) out[0] = s.v[1];
}
__global__ void k_big(Big s, float* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && s.v[0] < -1.0f) out[0] = s.v[511];
}

// four distinct kernels with 2 KB arguments, launched round robin (a frame's pass 1 / setup / walk / pass 2)
template <int I>
__global__ void k_big_n(Big s, float* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && s.v[0] < -1.0f) out[I] = s.v[511];
}

#define CHECK(x)                                                              \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));      \
            return 1;                                                         \
        }                                                                     \
    } while (0)

template <class F>
double per_call_us(hipStream_t s, F&& fn) {
    double best = 1e30;
    for (int rep = 0; rep < 7; ++rep) {
        if (hipStreamSynchronize(s) != hipSuccess) return -1.0;
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 64; ++i) fn();
        const auto t1 = std::chrono::steady_clock::now();
        const double us = std::chrono::duration<double, std::micro>(t1 - t0).count() / 64.0;
        best = us < best ? us : best;
    }
    return best;
}

int main() {
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float* out = nullptr;
    CHECK(hipMalloc(&out, 4));
    Small sm{};
    Big bg{};
    hipEvent_t ev;
    CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    hipEvent_t evt;
    CHECK(hipEventCreate(&evt));
    // warm-up: code objects loaded, queues created
    for (int i = 0; i < 100; ++i) {
        hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, sm, out);
        hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, bg, out);
    }
    CHECK(hipStreamSynchronize(s));
    const double small = per_call_us(s, [&] { hipLaunchKernelGGL(k_small, dim3(8160), dim3(256), 0, s, sm, out); });
    const double big = per_call_us(s, [&] { hipLaunchKernelGGL(k_big, dim3(8160), dim3(256), 0, s, bg, out); });
    const double rec = per_call_us(s, [&] { (void)hipEventRecord(ev, s); });
    const double rect = per_call_us(s, [&] { (void)hipEventRecord(evt, s); });
    const double gle = per_call_us(s, [&] { (void)hipGetLastError(); });
    int dev = 0;
    const double gd = per_call_us(s, [&] { (void)hipGetDevice(&dev); });
    // the band frame's count matrix to the host: an async copy into pinned memory vs a kernel writing it
    long long* dsrc = nullptr;
    long long* hpin = nullptr;
    CHECK(hipMalloc(&dsrc, 9 * 8 * 8));
    CHECK(hipHostMalloc((void**)&hpin, 9 * 8 * 8, hipHostMallocDefault));
    const double d2h = per_call_us(s, [&] { (void)hipMemcpyAsync(hpin, dsrc, 9 * 8 * 8, hipMemcpyDeviceToHost, s); });
    const double mset = per_call_us(s, [&] { (void)hipMemsetAsync(dsrc, 0, 9 * 8 * 8, s); });
    // 4 distinct kernels round robin (per launch), and the same through hipModuleLaunchKernel on function handles
    // looked up once (hipGetFuncBySymbol), the arguments passed as one buffer (HIP_LAUNCH_PARAM_BUFFER_POINTER)
    int rr = 0;
    const double rr4 = per_call_us(s, [&] {
        switch (rr++ & 3) {
            case 0: hipLaunchKernelGGL(k_big_n<0>, dim3(8160), dim3(256), 0, s, bg, out); break;
            case 1: hipLaunchKernelGGL(k_big_n<1>, dim3(8160), dim3(256), 0, s, bg, out); break;
            case 2: hipLaunchKernelGGL(k_big_n<2>, dim3(8160), dim3(256), 0, s, bg, out); break;
            default: hipLaunchKernelGGL(k_big_n<3>, dim3(8160), dim3(256), 0, s, bg, out); break;
        }
    });
    hipFunction_t fh[4];
    CHECK(hipGetFuncBySymbol(&fh[0], reinterpret_cast<const void*>(&k_big_n<0>)));
    CHECK(hipGetFuncBySymbol(&fh[1], reinterpret_cast<const void*>(&k_big_n<1>)));
    CHECK(hipGetFuncBySymbol(&fh[2], reinterpret_cast<const void*>(&k_big_n<2>)));
    CHECK(hipGetFuncBySymbol(&fh[3], reinterpret_cast<const void*>(&k_big_n<3>)));
    struct {
        Big b;
        float* o;
    } argbuf{bg, out};
    size_t argsz = sizeof(argbuf);
    void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &argbuf, HIP_LAUNCH_PARAM_BUFFER_SIZE, &argsz, HIP_LAUNCH_PARAM_END};
    rr = 0;
    const double mod4 = per_call_us(s, [&] {
        (void)hipModuleLaunchKernel(fh[rr++ & 3], 8160, 1, 1, 256, 1, 1, 0, s, nullptr, cfg);
    });
    // librsd's per-call host helpers: one getenv of a tuning variable, the "%f" round trip of RAY_CONE_SPREAD
    volatile const char* sink = nullptr;
    const double genv = per_call_us(s, [&] { sink = std::getenv("RSD_PASS2_LOOP"); });
    volatile float fs = 0.0f;
    const double spread = per_call_us(s, [&] {
        char buf[64];
        std::snprintf(buf, sizeof(buf), "%f", (double)std::atan(0.0012f));
        fs = std::strtof(buf, nullptr);
    });
    (void)sink;
    (void)fs;
    CHECK(hipStreamSynchronize(s));
    std::printf("{\"launch_us_args64\": %.2f, \"launch_us_args2048\": %.2f, \"event_record_us\": %.2f, "
                "\"event_record_timing_us\": %.2f, \"get_last_error_us\": %.3f, \"get_device_us\": %.3f, "
                "\"memcpy_d2h_pinned_576B_us\": %.2f, \"memset_576B_us\": %.2f, \"getenv_us\": %.3f, "
                "\"cone_spread_format_us\": %.3f, \"launch_us_4kernels_args2048\": %.2f, "
                "\"module_launch_us_4kernels_args2048\": %.2f}\n",
                small, big, rec, rect, gle, gd, d2h, mset, genv, spread, rr4, mod4);
    return 0;
}
