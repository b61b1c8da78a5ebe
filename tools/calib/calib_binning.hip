// calib_binning.hip -- what the binning step of a treelet-scheduled traversal
// ("Curve data in LDS") costs per metric frame on MI355X, with no
// traversal at all.  A treelet scheduler suspends every ray at every treelet it
// enters and regroups the suspension records by treelet before the LDS-resident
// pass (tools/treelet_sim.py on the metric row's real rays: 85M suspensions per
// frame at 32 KB treelets, 41k treelets).  Two ways to regroup them are timed:
//
//   counting sort : producer writes a 16-B record + atomicAdd(count[tid]);
//                   one-block exclusive scan; scatter with atomicAdd(cursor[tid])
//   radix sort    : hipcub::DeviceRadixSort::SortPairs on (tid, index), 17-bit keys
//
// plus the consumer's read of the grouped records.  Treelet ids are uniform
// random here (the real ones are skewed -- 130 to 1,700 rays per treelet and
// round -- which only adds atomic contention, so these are lower bounds).
// Prints one JSON line.  usage: calib_binning [n_records] [n_bins] [rounds]
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                      \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// producer: one suspension record per thread (ray index, treelet, entry t0/t1) + the bin count
__global__ void k_emit(uint32_t n, uint32_t bins, uint32_t salt, uint4* rec, uint32_t* keys, uint32_t* count) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t tid = hash32(i ^ salt) % bins;
    rec[i] = make_uint4(i, tid, __float_as_uint(0.5f), __float_as_uint(2.0f));
    keys[i] = tid;
    atomicAdd(&count[tid], 1u);
}

// one block: exclusive scan of the bin counts into offsets, cursors cleared
__global__ void k_scan(uint32_t bins, uint32_t* count, uint32_t* off, uint32_t* cursor) {
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x, per = (bins + 1023) / 1024, lo = t * per, hi = min(bins, lo + per);
    uint32_t s = 0;
    for (uint32_t b = lo; b < hi; ++b) s += count[b];
    part[t] = s;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint32_t v = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = part[t] - s;
    for (uint32_t b = lo; b < hi; ++b) {
        off[b] = run;
        run += count[b];
        count[b] = 0;
        cursor[b] = 0;
    }
}

__global__ void k_scatter(uint32_t n, const uint4* rec, const uint32_t* off, uint32_t* cursor, uint4* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 r = rec[i];
    out[off[r.y] + atomicAdd(&cursor[r.y], 1u)] = r;
}

// consumer: the grouped records read once (what the LDS pass would read)
__global__ void k_consume(uint32_t n, const uint4* in, uint32_t* sink) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 r = in[i];
    if (r.x == 0xFFFFFFFFu && r.y == r.z) sink[0] = r.w;  // never true: keeps the load
}

// radix path: sort (tid, index), then gather the records in sorted order
__global__ void k_gather(uint32_t n, const uint32_t* idx, const uint4* rec, uint4* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = rec[idx[i]];
}
__global__ void k_iota(uint32_t n, uint32_t* v) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = i;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atol(argv[1]) : 85000000u;
    const uint32_t bins = argc > 2 ? (uint32_t)atol(argv[2]) : 40975u;
    const int rounds = argc > 3 ? atoi(argv[3]) : 5;
    uint4 *rec, *out;
    uint32_t *keys, *keys2, *idx, *idx2, *count, *off, *cursor, *sink;
    CHK(hipMalloc(&rec, 16ull * n));
    CHK(hipMalloc(&out, 16ull * n));
    CHK(hipMalloc(&keys, 4ull * n));
    CHK(hipMalloc(&keys2, 4ull * n));
    CHK(hipMalloc(&idx, 4ull * n));
    CHK(hipMalloc(&idx2, 4ull * n));
    CHK(hipMalloc(&count, 4ull * bins));
    CHK(hipMalloc(&off, 4ull * bins));
    CHK(hipMalloc(&cursor, 4ull * bins));
    CHK(hipMalloc(&sink, 4));
    CHK(hipMemset(count, 0, 4ull * bins));
    int end_bit = 1;
    while ((1u << end_bit) < bins) ++end_bit;
    size_t tmp_bytes = 0;
    CHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys, keys2, idx, idx2, (int)n, 0, end_bit));
    void* tmp;
    CHK(hipMalloc(&tmp, tmp_bytes));
    const dim3 B(256), G((n + 255) / 256);
    hipEvent_t e[7];
    for (auto& x : e) CHK(hipEventCreate(&x));
    double t_emit = 0, t_scan = 0, t_scatter = 0, t_consume = 0, t_radix = 0, t_gather = 0;
    for (int r = -1; r < rounds; ++r) {  // round -1: warm-up
        CHK(hipEventRecord(e[0]));
        hipLaunchKernelGGL(k_emit, G, B, 0, 0, n, bins, 0x9E3779B9u * (r + 2), rec, keys, count);
        CHK(hipEventRecord(e[1]));
        hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, 0, bins, count, off, cursor);
        CHK(hipEventRecord(e[2]));
        hipLaunchKernelGGL(k_scatter, G, B, 0, 0, n, rec, off, cursor, out);
        CHK(hipEventRecord(e[3]));
        hipLaunchKernelGGL(k_consume, G, B, 0, 0, n, out, sink);
        CHK(hipEventRecord(e[4]));
        hipLaunchKernelGGL(k_iota, G, B, 0, 0, n, idx);
        CHK(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys, keys2, idx, idx2, (int)n, 0, end_bit));
        CHK(hipEventRecord(e[5]));
        hipLaunchKernelGGL(k_gather, G, B, 0, 0, n, idx2, rec, out);
        CHK(hipEventRecord(e[6]));
        CHK(hipEventSynchronize(e[6]));
        float ms[6];
        for (int k = 0; k < 6; ++k) CHK(hipEventElapsedTime(&ms[k], e[k], e[k + 1]));
        if (r >= 0) {
            t_emit += ms[0];
            t_scan += ms[1];
            t_scatter += ms[2];
            t_consume += ms[3];
            t_radix += ms[4];
            t_gather += ms[5];
        }
    }
    const double R = rounds;
    printf("{\"records\": %u, \"bins\": %u, \"key_bits\": %d, \"rounds\": %d, \"ms\": {\"emit_write_atomic\": %.3f, "
           "\"scan\": %.3f, \"scatter_atomic\": %.3f, \"consume_read\": %.3f, \"radix_sort_pairs\": %.3f, "
           "\"radix_gather\": %.3f}, \"counting_sort_total_ms\": %.3f, \"radix_total_ms\": %.3f}\n",
           n, bins, end_bit, rounds, t_emit / R, t_scan / R, t_scatter / R, t_consume / R, t_radix / R, t_gather / R,
           (t_emit + t_scan + t_scatter + t_consume) / R, (t_emit + t_radix + t_gather + t_consume) / R);
    return 0;
}
