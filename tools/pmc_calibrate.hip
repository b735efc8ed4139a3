// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// patterns of the traversal kernels (tools only, not part of libigx).
//
// MI355X_MICROARCH.md (HBM section) calibrates FETCH_SIZE only for wide
// coalesced streaming reads (it reports half the bytes).  The traversal reads
// scattered fixed-size records (16 B path-state columns, 48 B triangles,
// 64 B BVH2 nodes, 128 B 4-wide nodes), so this program launches one kernel
// per record size that reads a known number of random records from a 4 GiB
// table (far beyond the 256 MiB Infinity Cache: nearly every record is a miss)
// and one coalesced streaming read and write for reference.  Each launch reads
// `n` records; the expected number of distinct records is N (1 - exp(-n / N))
// for N records in the table.  Run under `rocprofv3 --pmc FETCH_SIZE` and
// `--pmc WRITE_SIZE` (separate passes); tools/profile_summary.py's
// `calibration` turns the counters into counter bytes / useful bytes.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/pmc_calibrate.hip -o tools/pmc_calibrate
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>

namespace {

__device__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// each lane reads one random record of F4 float4s (16 * F4 bytes)
template <int F4>
__global__ void __launch_bounds__(256) k_gather(const float4* __restrict__ table, unsigned long long records,
                                                 unsigned n, unsigned seed, float* __restrict__ out) {
    unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned long long r = ((unsigned long long)hash32(i * 2654435761U + seed) << 16 ^ hash32(i + seed * 7919U)) % records;
    const float4* p = table + r * F4;
    float s = 0;
#pragma unroll
    for (int k = 0; k < F4; ++k) {
        float4 v = p[k];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.0f) out[i] = s; // never true for a zeroed table: no store traffic
}

__global__ void __launch_bounds__(256) k_stream_read(const float4* __restrict__ a, size_t n, float* __restrict__ out) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    float s = 0;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.0f) out[0] = s;
}

__global__ void __launch_bounds__(256) k_stream_write(float4* __restrict__ a, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = make_float4(1, 2, 3, 4);
}

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

template <int F4>
void gather(const float4* table, size_t table_bytes, unsigned n, float* out) {
    unsigned long long records = table_bytes / (16ull * F4);
    double uniq = (double)records * (1.0 - std::exp(-(double)n / (double)records));
    hipLaunchKernelGGL(k_gather<F4>, dim3((n + 255) / 256), dim3(256), 0, 0, table, records, n, 17u, out);
    CHECK(hipDeviceSynchronize());
    std::printf("{\"kernel\": \"k_gather<%d>\", \"record_bytes\": %d, \"lanes\": %u, \"expected_unique_bytes\": %.0f}\n",
                F4, 16 * F4, n, uniq * 16 * F4);
}

} // namespace

int main() {
    const size_t table_bytes = 4ull << 30;
    float4* table;
    float* out;
    CHECK(hipMalloc(&table, table_bytes));
    CHECK(hipMalloc(&out, 64u << 20));
    CHECK(hipMemset(table, 0, table_bytes));
    CHECK(hipDeviceSynchronize());
    const unsigned n = 1u << 22; // 4 M records per launch
    gather<1>(table, table_bytes, n, out);
    gather<3>(table, table_bytes, n, out);
    gather<4>(table, table_bytes, n, out);
    gather<8>(table, table_bytes, n, out);
    const size_t sn = (1ull << 30) / 16; // 1 GiB streamed
    hipLaunchKernelGGL(k_stream_read, dim3(4096), dim3(256), 0, 0, table, sn, out);
    CHECK(hipDeviceSynchronize());
    std::printf("{\"kernel\": \"k_stream_read\", \"bytes\": %zu}\n", sn * 16);
    hipLaunchKernelGGL(k_stream_write, dim3(4096), dim3(256), 0, 0, table + sn, sn);
    CHECK(hipDeviceSynchronize());
    std::printf("{\"kernel\": \"k_stream_write\", \"bytes\": %zu}\n", sn * 16);
    CHECK(hipFree(table));
    CHECK(hipFree(out));
    return 0;
}
