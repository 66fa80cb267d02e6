// col_bench.hip — the pricing stream's access pattern alone: 256 workgroups
// x 8 waves walk NC columns of L doubles round-robin (a wave per column, 16
// dbl2 loads per lane in flight, as k_price), summing them.  Columns sit at a
// stride of L + PAD doubles, so PAD > 0 staggers the columns' starts across
// the HBM channels.  Prints the kernel time and the spread of workgroup end
// times (s_memrealtime).  Build:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/cb tools/col_bench.hip && /tmp/cb [NC=12288] [L=4096]
#include <hip/hip_runtime.h>

#include <algorithm>
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

__global__ __launch_bounds__(512) void k_cols(const double* __restrict__ A, long nc, long L2, long ld,
                                              double* __restrict__ out, unsigned long long* __restrict__ tend) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long stride = (long)gridDim.x * 8;
    double acc = 0.0;
    for (long j = (long)blockIdx.x * 8 + wave; j < nc; j += stride) {
        const dbl2* col = reinterpret_cast<const dbl2*>(A + j * ld);
        for (long k = lane; k < L2; k += 16 * 64) {
            dbl2 v[16];
#pragma unroll
            for (int t = 0; t < 16; ++t) v[t] = __builtin_nontemporal_load(&col[k + t * 64]);
#pragma unroll
            for (int t = 0; t < 16; ++t) acc += v[t].x + v[t].y;
        }
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    __syncthreads();
    if (threadIdx.x == 0) tend[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    if (lane == 0 && acc == 1234.5) out[0] = acc;
}

__global__ void k_t0(unsigned long long* t) { *t = __builtin_amdgcn_s_memrealtime(); }

int main(int argc, char** argv) {
    const long nc = argc > 1 ? atol(argv[1]) : 12288;
    const long L = argc > 2 ? atol(argv[2]) : 4096;
    const int grid = 256;
    double* A = nullptr;
    double* out = nullptr;
    unsigned long long *tend = nullptr, *t0 = nullptr;
    const long maxpad = 1024;
    CK(hipMalloc(&A, (size_t)nc * (L + maxpad) * 8));
    CK(hipMemset(A, 0, (size_t)nc * (L + maxpad) * 8));
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&tend, grid * 8));
    CK(hipMalloc(&t0, 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<unsigned long long> h(grid);
    for (long pad : {0L, 64L, 128L, 256L, 0L, 64L}) {
        const long ld = L + pad;
        float best = 1e9f;
        double spread = 0, p50 = 0;
        for (int r = 0; r < 20; ++r) {
            k_t0<<<1, 1>>>(t0);
            CK(hipEventRecord(e0));
            k_cols<<<grid, 512>>>(A, nc, L / 2, ld, out, tend);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) {
                best = ms;
                unsigned long long s0 = 0;
                CK(hipMemcpy(&s0, t0, 8, hipMemcpyDeviceToHost));
                CK(hipMemcpy(h.data(), tend, grid * 8, hipMemcpyDeviceToHost));
                std::sort(h.begin(), h.end());
                spread = (h[grid - 1] - h[0]) * 0.01;
                p50 = (h[grid / 2] - s0) * 0.01;
            }
        }
        const double gb = (double)nc * L * 8 / 1e9;
        std::printf("{\"pad_doubles\": %ld, \"us\": %.2f, \"TBps\": %.3f, \"wg_end_spread_us\": %.2f, \"wg_end_p50_us\": %.2f}\n",
                    pad, best * 1e3, gb / (best * 1e-3) / 1e3, spread, p50);
    }
    return 0;
}
