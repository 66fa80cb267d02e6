// stream_bench.hip — floor of a one-shot HBM read kernel of the FTRAN's shape
// (rows of 32 KiB, one wave per row, dot with a 32 KiB vector, per-wave result
// store, no cross-workgroup tail), against the same bytes read as long
// grid-stride streams.  Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/sb tools/stream_bench.hip
//   /tmp/sb [rows=4096] [L=4096]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double dbl2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

// one wave per row (R rows per wave), U dbl2 loads per lane per round trip
template <int U, int R, int NT = 1>
__global__ __launch_bounds__(512) void k_rows(const double* __restrict__ B, const double* __restrict__ a,
                                              double* __restrict__ out, long rows, long L) {
    const int lane = threadIdx.x & 63;
    const long w = (long)blockIdx.x * 8 + (threadIdx.x >> 6);
    const long L2 = L >> 1;
    const dbl2* ap = reinterpret_cast<const dbl2*>(a);
    for (int r = 0; r < R; ++r) {
        const long i = w * R + r;
        if (i >= rows) return;
        const dbl2* src = reinterpret_cast<const dbl2*>(B + i * L);
        double acc = 0.0;
        for (long k = lane; k < L2; k += U * 64) {
            dbl2 bv[U], av[U];
#pragma unroll
            for (int t = 0; t < U; ++t) {
                bv[t] = NT ? __builtin_nontemporal_load(&src[k + t * 64]) : src[k + t * 64];
                av[t] = ap[k + t * 64];
            }
#pragma unroll
            for (int t = 0; t < U; ++t) {
                acc = fma(bv[t].x, av[t].x, acc);
                acc = fma(bv[t].y, av[t].y, acc);
            }
        }
        for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
        if (lane == 0) out[i] = acc;
    }
}

// plain grid-stride sum over the whole buffer (the streaming ceiling)
__global__ __launch_bounds__(512) void k_flat(const double* __restrict__ B, double* __restrict__ out, long n2) {
    const dbl2* src = reinterpret_cast<const dbl2*>(B);
    double acc = 0.0;
    const long stride = (long)gridDim.x * blockDim.x;
    for (long k = (long)blockIdx.x * blockDim.x + threadIdx.x; k < n2; k += stride * 8) {
        dbl2 v[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = (k + t * stride < n2) ? __builtin_nontemporal_load(&src[k + t * stride]) : dbl2{0, 0};
#pragma unroll
        for (int t = 0; t < 8; ++t) acc += v[t].x + v[t].y;
    }
    if (acc == 12345.678) out[0] = acc;
}

template <typename F>
static float timeit(F f, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return 1000.f * ms / reps;  // us
}

int main(int argc, char** argv) {
    const long rows = argc > 1 ? atol(argv[1]) : 4096;
    const long L = argc > 2 ? atol(argv[2]) : 4096;
    const size_t bytes = (size_t)rows * L * 8;
    double *B, *a, *out, *flush;
    CK(hipMalloc(&B, bytes));
    CK(hipMalloc(&a, L * 8));
    CK(hipMalloc(&out, rows * 8));
    const size_t fb = (size_t)1 << 30;  // 1 GiB to evict the Infinity Cache between launches
    CK(hipMalloc(&flush, fb));
    CK(hipMemset(B, 0, bytes));
    CK(hipMemset(a, 0, L * 8));
    CK(hipMemset(flush, 0, fb));
    const int reps = 50;
    auto report = [&](const char* name, float us) {
        std::printf("{\"kernel\": \"%s\", \"rows\": %ld, \"L\": %ld, \"MB\": %.1f, \"us\": %.2f, \"TBps\": %.3f}\n", name,
                    rows, L, bytes / 1e6, us, bytes / (us * 1e-6) / 1e12);
    };
    // each launch preceded by a 1 GiB flush read (timed separately and subtracted)
    auto flushk = [&]() { hipLaunchKernelGGL(k_flat, dim3(2048), dim3(512), 0, 0, flush, out, (long)(fb / 16)); };
    const float tf = timeit(flushk, reps);
    auto rows1 = [&]() {
        flushk();
        hipLaunchKernelGGL((k_rows<16, 1>), dim3((rows + 7) / 8), dim3(512), 0, 0, B, a, out, rows, L);
    };
    report("rows U16 R1 (FTRAN shape), cold", timeit(rows1, reps) - tf);
    auto rows1w = [&]() { hipLaunchKernelGGL((k_rows<16, 1>), dim3((rows + 7) / 8), dim3(512), 0, 0, B, a, out, rows, L); };
    report("rows U16 R1 back-to-back", timeit(rows1w, reps));
    auto rows8 = [&]() {
        flushk();
        hipLaunchKernelGGL((k_rows<8, 1>), dim3((rows + 7) / 8), dim3(512), 0, 0, B, a, out, rows, L);
    };
    report("rows U8 R1, cold", timeit(rows8, reps) - tf);
    auto rows4 = [&]() {
        flushk();
        hipLaunchKernelGGL((k_rows<8, 4>), dim3((rows / 4 + 7) / 8), dim3(512), 0, 0, B, a, out, rows, L);
    };
    report("rows U8 R4 (long-lived waves), cold", timeit(rows4, reps) - tf);
    auto flat = [&]() {
        flushk();
        hipLaunchKernelGGL(k_flat, dim3(1024), dim3(512), 0, 0, B, out, (long)(bytes / 16));
    };
    report("flat grid-stride, cold", timeit(flat, reps) - tf);
    // default-policy rows: Infinity Cache residency of B between launches,
    // alone and behind a 3x-sized non-temporal stream (the pricing pass's A)
    auto rows8d = [&]() { hipLaunchKernelGGL((k_rows<8, 1, 0>), dim3((rows + 7) / 8), dim3(512), 0, 0, B, a, out, rows, L); };
    report("rows U8 R1 default policy, back-to-back", timeit(rows8d, reps));
    auto rows8dc = [&]() {
        flushk();
        hipLaunchKernelGGL((k_rows<8, 1, 0>), dim3((rows + 7) / 8), dim3(512), 0, 0, B, a, out, rows, L);
    };
    report("rows U8 R1 default policy, cold", timeit(rows8dc, reps) - tf);
    const long an2 = (long)(3 * bytes / 16);
    auto astream = [&]() { hipLaunchKernelGGL(k_flat, dim3(2048), dim3(512), 0, 0, flush, out, an2); };
    const float ta = timeit(astream, reps);
    auto rows8da = [&]() {
        astream();
        hipLaunchKernelGGL((k_rows<8, 1, 0>), dim3((rows + 7) / 8), dim3(512), 0, 0, B, a, out, rows, L);
    };
    report("rows U8 R1 default policy, behind a 3x nt stream", timeit(rows8da, reps) - ta);
    auto rows8na = [&]() {
        astream();
        hipLaunchKernelGGL((k_rows<8, 1, 1>), dim3((rows + 7) / 8), dim3(512), 0, 0, B, a, out, rows, L);
    };
    report("rows U8 R1 nt, behind a 3x nt stream", timeit(rows8na, reps) - ta);
    std::printf("{\"kernel\": \"3x nt stream\", \"us\": %.2f}\n", ta);
    std::printf("{\"kernel\": \"flush 1GiB\", \"us\": %.2f}\n", tf);
    return 0;
}
