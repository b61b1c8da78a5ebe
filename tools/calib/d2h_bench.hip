// Calibration (dev tool, GPU box): device-to-host copy paths for the tonemapped
// texture's 16.6 MB of log terms (one 1080p frame of doubles): pageable memory,
// pinned memory (hipHostMalloc default / non-coherent / hipHostRegister), whole
// or in 16 chunks, by hipMemcpyAsync or by a kernel storing into the pinned
// buffer (zero copy).  Prints ms per copy and GB/s.
// Build: hipcc -O2 --offload-arch=gfx950 -o d2h_bench d2h_bench.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

__global__ void k_store(const double* __restrict__ src, double* dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t n = 1920 * 1080, bytes = n * 8;
    double* d;
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(d, 1, bytes));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    std::vector<double> pageable(n);
    double *pin_def, *pin_nc, *pin_wc;
    CK(hipHostMalloc((void**)&pin_def, bytes, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&pin_nc, bytes, hipHostMallocNonCoherent));
    CK(hipHostMalloc((void**)&pin_wc, bytes, hipHostMallocMapped));
    std::vector<double> reg(n);
    CK(hipHostRegister(reg.data(), bytes, hipHostRegisterDefault));
    struct Case {
        const char* name;
        double* dst;
        int chunks;
        bool kernel;
    } cases[] = {{"pageable whole", pageable.data(), 1, false}, {"pageable 16 chunks", pageable.data(), 16, false},
                 {"pinned default whole", pin_def, 1, false},   {"pinned default 16 chunks", pin_def, 16, false},
                 {"pinned noncoherent whole", pin_nc, 1, false}, {"pinned noncoherent 16 chunks", pin_nc, 16, false},
                 {"registered whole", reg.data(), 1, false},   {"registered 16 chunks", reg.data(), 16, false},
                 {"kernel store to pinned default", pin_def, 1, true}, {"kernel store to pinned mapped", pin_wc, 1, true}};
    for (const Case& c : cases) {
        double best = 1e30;
        for (int rep = 0; rep < 6; ++rep) {
            CK(hipStreamSynchronize(s));
            const double t0 = now_ms();
            if (c.kernel) {
                double* dp = c.dst;
                CK(hipHostGetDevicePointer((void**)&dp, c.dst, 0));
                hipLaunchKernelGGL(k_store, dim3(1024), dim3(256), 0, s, d, dp, n);
            } else {
                const size_t per = (n + c.chunks - 1) / c.chunks;
                for (int k = 0; k < c.chunks; ++k) {
                    const size_t a = k * per, b = a + per < n ? a + per : n;
                    CK(hipMemcpyAsync(c.dst + a, d + a, (b - a) * 8, hipMemcpyDeviceToHost, s));
                }
            }
            CK(hipStreamSynchronize(s));
            const double t = now_ms() - t0;
            if (t < best) best = t;
        }
        // CPU read of the landed data (sum), to expose uncached host memory
        const double t1 = now_ms();
        double acc = 0;
        for (size_t i = 0; i < n; ++i) acc += c.dst[i];
        const double tr = now_ms() - t1;
        printf("%-32s %.3f ms  %.1f GB/s   cpu read %.3f ms (%g)\n", c.name, best, bytes / best / 1e6, tr, acc);
    }
    return 0;
}
