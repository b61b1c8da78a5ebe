// calib_tcp.hip -- is random 64-B record fetching limited per CU by per-lane
// line lookups (vector L1 / TA), independent of where the lines live?
//
// For tables that fit L2 (2 MiB), the Infinity Cache (64 MiB) and HBM (2 GiB):
//   lane64 : each lane fetches its own random 64-B record with 4 x 16-B loads
//            (the traversal kernels' pattern: 4 lookups per lane per record)
//   quad64 : the 4 lanes of a quad fetch the 4 records of the quad together:
//            load j reads record (quad lane j) as 4 x 16 B spread over the quad
//            (one line per quad per load), then a 4x4 in-quad transpose with
//            DPP gives every lane its own record
//   lane16 : one random 16-B load per lane (1 lookup per lane)
// Prints time per million lanes and lanes/cycle/CU (clock from hipDeviceProp).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                              \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
            exit(1);                                                        \
        }                                                                   \
    } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// quad_perm DPP controls: lane i of a quad reads lane sel[i]
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
#define QP(a, b, c, d) ((a) | ((b) << 2) | ((c) << 4) | ((d) << 6))

// 4x4 transpose in a quad: in[j] = piece (lane&3) of record j; out[k] = piece k of record (lane&3)
__device__ __forceinline__ void quad_transpose(float in[4], float out[4]) {
    const int l = threadIdx.x & 3;
    // stage 1: exchange with lane ^ 1 (swap odd/even record slots)
    float s0 = dpp<QP(1, 0, 3, 2)>(in[l & 1 ? 0 : 1]);
    float s1 = dpp<QP(1, 0, 3, 2)>(in[l & 1 ? 2 : 3]);
    float a0 = (l & 1) ? s0 : in[0], a1 = (l & 1) ? in[1] : s0;
    float a2 = (l & 1) ? s1 : in[2], a3 = (l & 1) ? in[3] : s1;
    // stage 2: exchange with lane ^ 2
    float t0 = dpp<QP(2, 3, 0, 1)>((l & 2) ? a0 : a2);
    float t1 = dpp<QP(2, 3, 0, 1)>((l & 2) ? a1 : a3);
    out[0] = (l & 2) ? t0 : a0;
    out[1] = (l & 2) ? t1 : a1;
    out[2] = (l & 2) ? a2 : t0;
    out[3] = (l & 2) ? a3 : t1;
}

__global__ __launch_bounds__(256) void k_lane64(const float4* __restrict__ t, uint32_t n_rec, uint32_t n, uint32_t seed,
                                                float* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4* p = t + (size_t)(hash32(i ^ seed) % n_rec) * 4;
    float4 a = p[0], b = p[1], c = p[2], d = p[3];
    out[i] = (a.x + b.y) + (c.z + d.w);
}

__global__ __launch_bounds__(256) void k_lane16(const float4* __restrict__ t, uint32_t n_rec, uint32_t n, uint32_t seed,
                                                float* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float4 a = t[(size_t)(hash32(i ^ seed) % n_rec) * 4];
    out[i] = a.x + a.w;
}

__global__ __launch_bounds__(256) void k_quad64(const float4* __restrict__ t, uint32_t n_rec, uint32_t n, uint32_t seed,
                                                float* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;  // n is a multiple of 256: whole quads active
    const uint32_t q = i & ~3u, l = i & 3u;
    float4 piece[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t rec = hash32((q + j) ^ seed) % n_rec;  // record of quad lane j
        piece[j] = t[(size_t)rec * 4 + l];              // piece l of it
    }
    float ix[4], iy[4], iz[4], iw[4], ox[4], oy[4], oz[4], ow[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        ix[j] = piece[j].x; iy[j] = piece[j].y; iz[j] = piece[j].z; iw[j] = piece[j].w;
    }
    quad_transpose(ix, ox);
    quad_transpose(iy, oy);
    quad_transpose(iz, oz);
    quad_transpose(iw, ow);
    // own record: piece k = (ox[k], oy[k], oz[k], ow[k]); same checksum as k_lane64
    out[i] = (ox[0] + oy[1]) + (oz[2] + ow[3]);
}

int main() {
    int dev = 0;
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, dev));
    const double clk_hz = prop.clockRate * 1e3;
    const int n_cu = prop.multiProcessorCount;
    const uint32_t n = 1u << 24;
    const size_t max_bytes = (size_t)2 << 30;
    float4* t;
    float *o1, *o2;
    CHK(hipMalloc(&t, max_bytes));
    // distinct values so the checksums compare the two fetch forms
    {
        size_t n4 = max_bytes / 16;
        float4* h = (float4*)malloc(16 << 20);
        for (size_t k = 0; k < (1u << 20); ++k) h[k] = make_float4(k * 1.0f, k * 2.0f, k * 3.0f, k * 4.0f);
        for (size_t off = 0; off < n4; off += (1u << 20)) CHK(hipMemcpy(t + off, h, 16 << 20, hipMemcpyHostToDevice));
        free(h);
    }
    CHK(hipMalloc(&o1, (size_t)n * 4));
    CHK(hipMalloc(&o2, (size_t)n * 4));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    const size_t sizes[3] = {(size_t)2 << 20, (size_t)64 << 20, max_bytes};
    const char* names[3] = {"L2 (2 MiB)", "MALL (64 MiB)", "HBM (2 GiB)"};
    printf("{\"clock_MHz\": %.0f, \"cus\": %d, \"lanes\": %u, \"rows\": [\n", clk_hz / 1e6, n_cu, n);
    for (int s = 0; s < 3; ++s) {
        uint32_t n_rec = (uint32_t)(sizes[s] / 64);
        float ms[3];
        for (int k = 0; k < 3; ++k) {
            auto go = [&] {
                if (k == 0) hipLaunchKernelGGL(k_lane64, dim3(n / 256), dim3(256), 0, 0, t, n_rec, n, 7u, o1);
                if (k == 1) hipLaunchKernelGGL(k_quad64, dim3(n / 256), dim3(256), 0, 0, t, n_rec, n, 7u, o2);
                if (k == 2) hipLaunchKernelGGL(k_lane16, dim3(n / 256), dim3(256), 0, 0, t, n_rec, n, 7u, o1);
            };
            go();
            CHK(hipDeviceSynchronize());
            CHK(hipEventRecord(a));
            for (int r = 0; r < 5; ++r) go();
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            CHK(hipEventElapsedTime(&ms[k], a, b));
            ms[k] /= 5;
        }
        // checksum equality: lane64 and quad64 computed the same per-lane value
        hipLaunchKernelGGL(k_lane64, dim3(n / 256), dim3(256), 0, 0, t, n_rec, n, 7u, o1);
        CHK(hipDeviceSynchronize());
        float* h1 = (float*)malloc((size_t)n * 4);
        float* h2 = (float*)malloc((size_t)n * 4);
        CHK(hipMemcpy(h1, o1, (size_t)n * 4, hipMemcpyDeviceToHost));
        CHK(hipMemcpy(h2, o2, (size_t)n * 4, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (uint32_t k = 0; k < n; ++k) bad += h1[k] != h2[k];
        free(h1);
        free(h2);
        auto lpc = [&](float m) { return (double)n / (m * 1e-3 * clk_hz) / n_cu; };
        printf("  {\"table\": \"%s\", \"lane64_ms\": %.4f, \"quad64_ms\": %.4f, \"lane16_ms\": %.4f, "
               "\"lane64_lanes_per_cyc_cu\": %.3f, \"quad64_lanes_per_cyc_cu\": %.3f, \"lane16_lanes_per_cyc_cu\": %.3f, "
               "\"quad_mismatch\": %zu}%s\n",
               names[s], ms[0], ms[1], ms[2], lpc(ms[0]), lpc(ms[1]), lpc(ms[2]), bad, s < 2 ? "," : "");
    }
    printf("]}\n");
    return 0;
}
