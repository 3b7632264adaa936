// Dependent-accumulator MFMA chains at one wave per SIMD (development probe): the
// split32 decoder (K7t) accumulates each 32x32 block as one chain of 3 x NK
// dependent v_mfma_f32_32x32x16_f16; this measures the rate of NACC interleaved
// chains per wave (1: every MFMA waits on the previous one) on random operands.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_chain.cpp -o tools/mfma_chain.bin
#include <hip/hip_runtime.h>

#include <cstdio>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256) void chain(int iters, float* out) {
    const unsigned seed = (blockIdx.x * 256u + threadIdx.x) * 2654435761u;
    h8 a, b;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const unsigned r = seed ^ (t * 0x9e3779b9u);
        a[t] = (_Float16)((float)((r >> 8) & 0xffff) / 65536.f - 0.5f);
        b[t] = (_Float16)((float)((r >> 3) & 0xffff) / 65536.f - 0.5f);
    }
    f16v c[NACC] = {};
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) c[k % NACC] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c[k % NACC], 0, 0, 0);
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < NACC; ++q)
#pragma unroll
        for (int e = 0; e < 16; ++e) s += c[q][e];
    if (s == 12345.678f) out[0] = s;
}

template <int NACC>
void run(float* d, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256;   // one workgroup of 4 waves per CU: one wave per SIMD
    for (int w = 0; w < 40; ++w) hipLaunchKernelGGL(chain<NACC>, dim3(blocks), dim3(256), 0, 0, iters, d);
    hipEventRecord(e0, 0);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(chain<NACC>, dim3(blocks), dim3(256), 0, 0, iters, d);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = (double)reps * blocks * 4 * iters * 4 * 32.0 * 32 * 16 * 2;
    printf("{\"chains_per_wave\": %d, \"waves_per_simd\": 1, \"f16_tflops\": %.1f}\n", NACC, flop / (ms * 1e-3) / 1e12);
}

int main() {
    float* d;
    hipMalloc(&d, 4);
    run<1>(d, 20000);
    run<2>(d, 20000);
    run<4>(d, 20000);
    run<1>(d, 20000);
    return 0;
}
