// GroupNorm micro-benchmark (development tool): the U-Net's GroupNorm shapes
// (64^2 x 128 with a 2-slab split-K source, 32^2 x 256 with 4 slabs + residual,
// plain 64^2 x 256 concat) through cfd::launch_gn at a given batch; prints time and
// the bandwidth over the algorithmic bytes.
//   hipcc -O2 --offload-arch=gfx950 -std=c++17 -Iinclude tools/gnbench.cpp -Lconfild_amd/lib -lconfild_hip \
//         -Wl,-rpath,'$ORIGIN/../confild_amd/lib' -o tools/gnbench.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../confild_amd/csrc/unet_kernels.hpp"

struct Shape {
    const char* name;
    int HW, C1, C2, ksplits, kres, kx;
};
static const Shape SHAPES[] = {
    {"64^2 x128 k2 (GN2)", 4096, 128, 0, 2, 0, 0},
    {"64^2 x128 k2 res kx (GN1)", 4096, 128, 0, 2, 1, 1},
    {"64^2 x128+128 k2 res kx", 4096, 128, 128, 2, 1, 1},
    {"32^2 x256 k4 (GN2)", 1024, 256, 0, 4, 0, 0},
    {"32^2 x256 k4 res kx", 1024, 256, 0, 4, 1, 1},
    {"64^2 x256+128 plain", 4096, 256, 128, 0, 0, 0},
    {"8^2 x512 k16 (GN2)", 64, 512, 0, 16, 0, 0},
};

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 8;
    hipStream_t st;
    hipStreamCreate(&st);
    for (const Shape& s : SHAPES) {
        const int Ct = s.C1 + s.C2;
        const size_t n1 = (size_t)B * s.HW * s.C1, n2 = (size_t)B * s.HW * s.C2, nt = (size_t)B * s.HW * Ct;
        const size_t slabs = s.ksplits ? s.ksplits : 1;
        std::vector<float> h(std::max(n1 * slabs, n2) + 16);
        for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 500.f - 1.f;
        float *src1, *src2 = nullptr, *res, *kx, *out, *ss, *gamma, *beta, *bias;
        double* part;
        hipMalloc(&src1, n1 * slabs * 4);
        hipMemcpy(src1, h.data(), n1 * slabs * 4, hipMemcpyHostToDevice);
        if (s.C2) {
            hipMalloc(&src2, n2 * 4);
            hipMemcpy(src2, h.data(), n2 * 4, hipMemcpyHostToDevice);
        }
        hipMalloc(&res, n1 * 4);
        hipMemcpy(res, h.data(), n1 * 4, hipMemcpyHostToDevice);
        hipMalloc(&kx, n1 * 4);
        hipMalloc(&out, nt * 4);
        hipMalloc(&ss, (size_t)B * Ct * 8);
        hipMalloc(&gamma, Ct * 4);
        hipMalloc(&beta, Ct * 4);
        hipMalloc(&bias, Ct * 4);
        hipMemcpy(gamma, h.data(), Ct * 4, hipMemcpyHostToDevice);
        hipMemcpy(beta, h.data() + 7, Ct * 4, hipMemcpyHostToDevice);
        hipMemcpy(bias, h.data() + 3, Ct * 4, hipMemcpyHostToDevice);
        hipMalloc(&part, (size_t)B * cfd::kGnMaxChunks * 32 * 2 * 8);
        cfd::GnArgs g{};
        g.src1 = src1;
        g.src2 = src2;
        g.gamma = gamma;
        g.beta = beta;
        g.part = part;
        g.ss = ss;
        g.out = out;
        g.C1 = s.C1;
        g.C2 = s.C2;
        g.Ctot = Ct;
        g.HW = s.HW;
        g.eps = 1e-5f;
        g.silu = 1;
        if (s.ksplits) {
            g.kpart = src1;
            g.ksplits = s.ksplits;
            g.kbias = bias;
            g.kres = s.kres ? res : nullptr;
            g.kx = s.kx ? kx : nullptr;
        }
        double bytes = (double)nt * 4 /*out*/ + (s.ksplits ? (double)n1 * 4 * s.ksplits + (s.kres ? n1 * 4.0 : 0) +
                                                                 (s.kx ? n1 * 4.0 : 0) + n2 * 4.0
                                                           : nt * 4.0);
        for (int w = 0; w < 5; ++w) cfd::launch_gn(g, B, st);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        const int it = 50;
        hipEventRecord(e0, st);
        for (int i = 0; i < it; ++i) cfd::launch_gn(g, B, st);
        hipEventRecord(e1, st);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1e3 / it;
        printf("%-28s B=%2d  %7.2f us  %6.1f MB  %5.2f TB/s\n", s.name, B, us, bytes / 1e6, bytes / (us * 1e-6) / 1e12);
        hipFree(src1);
        if (src2) hipFree(src2);
        hipFree(res);
        hipFree(kx);
        hipFree(out);
        hipFree(ss);
        hipFree(gamma);
        hipFree(beta);
        hipFree(bias);
        hipFree(part);
    }
    return 0;
}
