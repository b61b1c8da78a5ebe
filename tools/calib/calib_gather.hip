// calib_gather.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE against known
// byte counts for the access patterns of the traversal kernels, and measures the
// achievable bandwidth of random record gathers (the realistic ceiling for BVH
// traversal, which reads 64-B node and primitive records at random addresses).
//
//   k_stream    : coalesced 16 B/lane streaming read of the whole table
//   k_gather64  : one random 64-B record per lane (4 x 16-B loads), like a node fetch
//   k_gather32  : one random 32-B half record per lane (2 x 16-B loads)
//   k_gather128 : one random 128-B record pair per lane (8 x 16-B loads)
//
// Table = 2 GiB (far beyond the 256 MiB Infinity Cache), indices are a seeded
// hash, so every record read is an HBM read.  Prints one JSON line with each
// kernel's algorithmic bytes and event-timed GB/s; run it under rocprofv3 --pmc
// to read the counters against the same launches.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                             \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

__global__ void k_stream(const float4* __restrict__ t, size_t n16, float* out) {
    float acc = 0.0f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = t[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 1234.5f) out[0] = acc;  // keeps the loads alive, never true for zeroed data
}

template <int NV>  // 16-B loads per record
__global__ void k_gather(const float4* __restrict__ t, uint32_t n_rec, uint32_t n, uint32_t seed, float* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t r = hash32(i ^ seed) % n_rec;
    const float4* p = t + (size_t)r * NV;
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        float4 v = p[k];
        acc += v.x + v.y + v.z + v.w;
    }
    out[i] = acc;
}

int main(int argc, char** argv) {
    const size_t table_bytes = (size_t)2 << 30;
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 24);  // lanes per gather launch
    float4* t;
    float* out;
    CHK(hipMalloc(&t, table_bytes));
    CHK(hipMemset(t, 0, table_bytes));
    CHK(hipMalloc(&out, (size_t)n * 4));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    auto timeit = [&](auto launch, int reps) {
        launch();  // warm
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) launch();
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        return ms / reps;
    };
    const int reps = 5;
    size_t n16 = table_bytes / 16;
    float ms_s = timeit([&] { hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, t, n16, out); }, reps);
    uint32_t nb = (n + 255) / 256;
    float ms_32 = timeit([&] {
        hipLaunchKernelGGL(k_gather<2>, dim3(nb), dim3(256), 0, 0, t, (uint32_t)(table_bytes / 32), n, 1u, out);
    }, reps);
    float ms_64 = timeit([&] {
        hipLaunchKernelGGL(k_gather<4>, dim3(nb), dim3(256), 0, 0, t, (uint32_t)(table_bytes / 64), n, 2u, out);
    }, reps);
    float ms_128 = timeit([&] {
        hipLaunchKernelGGL(k_gather<8>, dim3(nb), dim3(256), 0, 0, t, (uint32_t)(table_bytes / 128), n, 3u, out);
    }, reps);
    auto gbs = [](double bytes, float ms) { return bytes / (ms * 1e-3) / 1e9; };
    printf("{\"table_bytes\": %zu, \"lanes\": %u, "
           "\"stream\": {\"read_bytes\": %zu, \"ms\": %.4f, \"GBps\": %.1f}, "
           "\"gather32\": {\"read_bytes\": %zu, \"write_bytes\": %zu, \"ms\": %.4f, \"GBps_read\": %.1f}, "
           "\"gather64\": {\"read_bytes\": %zu, \"write_bytes\": %zu, \"ms\": %.4f, \"GBps_read\": %.1f}, "
           "\"gather128\": {\"read_bytes\": %zu, \"write_bytes\": %zu, \"ms\": %.4f, \"GBps_read\": %.1f}}\n",
           table_bytes, n, table_bytes, ms_s, gbs((double)table_bytes, ms_s), (size_t)n * 32, (size_t)n * 4, ms_32,
           gbs((double)n * 32, ms_32), (size_t)n * 64, (size_t)n * 4, ms_64, gbs((double)n * 64, ms_64),
           (size_t)n * 128, (size_t)n * 4, ms_128, gbs((double)n * 128, ms_128));
    return 0;
}
