// Checks that a butterfly of DPP / permlane moves pairs lanes exactly as the
// __shfl_xor butterfly (offsets 32, 16, 8, 4, 2, 1) does, so a wave sum built
// from it has the same bits (spx_common.h wave_sum).  Prints mismatches.
//   hipcc --offload-arch=gfx950 -O3 tools/dpp_sum_check.hip -o /tmp/dpp_sum_check && /tmp/dpp_sum_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

__device__ __forceinline__ double xor_shfl(double v, int off) { return __shfl_xor(v, off, 64); }

template <int CTRL, int RM, int BM>
__device__ __forceinline__ double dppd(double old, double v) {
    const long long o = __double_as_longlong(old), b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp((int)o, (int)b, CTRL, RM, BM, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), CTRL, RM, BM, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double swap32(double v) {
    const int lane = threadIdx.x & 63;
    const long long b = __double_as_longlong(v);
    auto lo = __builtin_amdgcn_permlane32_swap((int)b, (int)b, false, false);
    auto hi = __builtin_amdgcn_permlane32_swap((int)(b >> 32), (int)(b >> 32), false, false);
    const int l = lane < 32 ? lo[1] : lo[0];
    const int h = lane < 32 ? hi[1] : hi[0];
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)h << 32) | (unsigned)l));
}
__device__ __forceinline__ double swap16(double v) {
    const int lane = threadIdx.x & 63;
    const long long b = __double_as_longlong(v);
    auto lo = __builtin_amdgcn_permlane16_swap((int)b, (int)b, false, false);
    auto hi = __builtin_amdgcn_permlane16_swap((int)(b >> 32), (int)(b >> 32), false, false);
    const bool odd = (lane >> 4) & 1;
    const int l = odd ? lo[0] : lo[1];
    const int h = odd ? hi[0] : hi[1];
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)h << 32) | (unsigned)l));
}
// partner values for each offset, DPP forms (variant v for xor 4)
template <int V>
__device__ __forceinline__ double partner(double v, int off) {
    switch (off) {
        case 32: return swap32(v);
        case 16: return swap16(v);
        case 8: return dppd<0x128, 0xF, 0xF>(v, v);  // row_ror:8
        case 4: {
            if (V == 0) {  // row_shl:4 into banks 0,2; row_shr:4 into banks 1,3
                double t = dppd<0x104, 0xF, 0x5>(v, v);
                return dppd<0x114, 0xF, 0xA>(t, v);
            } else {  // the other direction
                double t = dppd<0x114, 0xF, 0x5>(v, v);
                return dppd<0x104, 0xF, 0xA>(t, v);
            }
        }
        case 2: return dppd<0x4E, 0xF, 0xF>(v, v);
        default: return dppd<0xB1, 0xF, 0xF>(v, v);
    }
}
template <int V>
__global__ void k(const double* in, double* out, int* pairs) {
    const int lane = threadIdx.x;
    double a = in[lane], b = a;
    for (int off = 32; off > 0; off >>= 1) {
        const double pa = xor_shfl(a, off);
        const double pb = partner<V>(b, off);
        // which lane did the DPP form pair with?  (tag values: lane index)
        const double tag = partner<V>((double)lane, off);
        pairs[(31 - __builtin_clz(off)) * 64 + lane] = (int)tag;
        a += pa;
        b += pb;
    }
    out[lane] = a;
    out[64 + lane] = b;
}
int main() {
    double h[64];
    srand(7);
    for (int i = 0; i < 64; ++i) h[i] = (rand() / (double)RAND_MAX - 0.5) * (1 << (i % 20));
    double *din, *dout;
    int* dp;
    hipMalloc(&din, 64 * 8);
    hipMalloc(&dout, 128 * 8);
    hipMalloc(&dp, 6 * 64 * 4);
    hipMemcpy(din, h, 64 * 8, hipMemcpyHostToDevice);
    for (int V = 0; V < 2; ++V) {
        if (V == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, din, dout, dp);
        else hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, din, dout, dp);
        double o[128];
        int pr[6 * 64];
        hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
        hipMemcpy(pr, dp, sizeof(pr), hipMemcpyDeviceToHost);
        int bad_pair = 0, bad_bits = 0;
        for (int s = 0; s < 6; ++s)
            for (int l = 0; l < 64; ++l)
                if (pr[s * 64 + l] != (l ^ (1 << s))) ++bad_pair;
        for (int l = 0; l < 64; ++l)
            if (memcmp(&o[l], &o[64 + l], 8) != 0) ++bad_bits;
        printf("variant %d: pairing mismatches %d, bit mismatches %d\n", V, bad_pair, bad_bits);
    }
    return 0;
}
