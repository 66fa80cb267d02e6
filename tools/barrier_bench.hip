// Grid-barrier cost on one MI355X: a cooperative launch (one workgroup per
// CU) that runs N barriers, timed with hipEvents; variants of the barrier.
//   hipcc --offload-arch=gfx950 -O3 -I../simplex_method_gpu_amd/csrc tools/barrier_bench.hip -o tools/barrier_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#include "spx_grid.h"

using namespace spx;

template <int VARIANT>
__global__ __launch_bounds__(512) void k_bar(LoopState* ls, int nbar, double* sink) {
    __shared__ int s_ok;
    uint32_t target = 0;
    double acc = 0.0;
    for (int b = 0; b < nbar; ++b) {
        if constexpr (VARIANT == 1) {  // a partial store per workgroup before the barrier
            if (threadIdx.x == 0) st_agent(&sink[blockIdx.x], acc + b);
        }
        target += gridDim.x;
        if (!grid_sync(ls, target, &s_ok)) return;
        if constexpr (VARIANT == 1) {  // every workgroup reads all partials after it
            double s = 0.0;
            for (int g = threadIdx.x; g < (int)gridDim.x; g += 512) s += ld_agent(&sink[g]);
            acc += s;
        }
    }
    if (threadIdx.x == 0 && acc == -1.0) sink[0] = acc;
}

template <int V>
float run(int cus, int nbar, LoopState* ls, double* sink) {
    hipMemset(ls, 0, sizeof(LoopState));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    void* args[] = {&ls, &nbar, &sink};
    hipEventRecord(e0, 0);
    hipLaunchCooperativeKernel(reinterpret_cast<const void*>(&k_bar<V>), dim3(cus), dim3(512), args, 0, 0);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main(int argc, char** argv) {
    int dev = 0;
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, dev);
    const int cus = prop.multiProcessorCount;
    LoopState* ls;
    double* sink;
    hipMalloc(&ls, sizeof(LoopState));
    hipMalloc(&sink, sizeof(double) * 1024);
    for (int g : {cus, cus / 2, cus / 4, 32, 8}) {
        for (int rep = 0; rep < 2; ++rep) {
            const float t1 = run<0>(g, 10, ls, sink);
            const float t2 = run<0>(g, 1010, ls, sink);
            const float u1 = run<1>(g, 10, ls, sink);
            const float u2 = run<1>(g, 1010, ls, sink);
            if (rep) printf("{\"workgroups\": %d, \"barrier_us\": %.3f, \"barrier_plus_partials_us\": %.3f}\n", g,
                            1e3 * (t2 - t1) / 1000.0, 1e3 * (u2 - u1) / 1000.0);
        }
    }
    return 0;
}
