// Convolution micro-benchmark (development tool): the U-Net's convolution
// shapes at config B (B = 8, 64x64) through the shipped planner/kernel
// (cfd::plan_conv + cfd::launch_conv, K1s) and through the K1x variants
// (cfd::launch_conv_x), on identical split-f16 operands.  Prints per shape the
// time of each, its TFLOP/s, and the max |difference| against K1s relative to
// max |K1s| (both are fp32-accurate; differences are summation-order rounding).
//
//   hipcc -O2 --offload-arch=gfx950 -std=c++17 -Iinclude tools/convbench.cpp \
//         -Lconfild_amd/lib -lconfild_hip -Wl,-rpath,$PWD/confild_amd/lib -o build/convbench
//   build/convbench [variant ...]          (default: all variants)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../confild_amd/csrc/unet_kernels.hpp"

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

namespace cfd {
int launch_conv_x(const ConvArgs& a, int variant, int splits, hipStream_t st);
int conv_h_tw(const ConvArgs& a);
}

struct Shape {
    const char* name;
    int B, Hin, Win, C1, C2, Cout, ks, stride, up;
};

static const Shape SHAPES[] = {
    {"L0 conv 128->128", 8, 64, 64, 128, 0, 128, 3, 1, 0},
    {"L0 out 256+128->128", 8, 64, 64, 256, 128, 128, 3, 1, 0},
    {"L0 out 128+128->128", 8, 64, 64, 128, 128, 128, 3, 1, 0},
    {"L1 up 256->256 (32->64)", 8, 32, 32, 256, 0, 256, 3, 1, 1},
    {"L0 down 128 s2", 8, 64, 64, 128, 0, 128, 3, 2, 0},
    {"L1 conv 256->256", 8, 32, 32, 256, 0, 256, 3, 1, 0},
    {"L1 out 384+256->256", 8, 32, 32, 384, 256, 256, 3, 1, 0},
    {"L2 conv 384->384", 8, 16, 16, 384, 0, 384, 3, 1, 0},
    {"L3 conv 512->512", 8, 8, 8, 512, 0, 512, 3, 1, 0},
    {"L0 skip1x1 384->128", 8, 64, 64, 256, 128, 128, 1, 1, 0},
    {"L1 skip1x1 640->256", 8, 32, 32, 384, 256, 256, 1, 1, 0},
    {"L2 skip1x1 768->384", 8, 16, 16, 384, 384, 384, 1, 1, 0},
    {"L3 skip1x1 1024->512", 8, 8, 8, 512, 512, 512, 1, 1, 0},
    {"L1 proj 256->256", 8, 32, 32, 256, 0, 256, 1, 1, 0},
    {"L3 conv 1024->512", 8, 8, 8, 1024, 0, 512, 3, 1, 0},
    {"L2 conv 768->384", 8, 16, 16, 768, 0, 384, 3, 1, 0},
    {"L2 conv 896->384", 8, 16, 16, 896, 0, 384, 3, 1, 0},
    {"L2 conv 640->384", 8, 16, 16, 640, 0, 384, 3, 1, 0},
    {"L2 up 384->384", 8, 8, 8, 384, 0, 384, 3, 1, 1},
    {"L3 qkv 512->1536", 8, 8, 8, 512, 0, 1536, 1, 1, 0},
    {"L2 qkv 384->1152", 8, 16, 16, 384, 0, 1152, 1, 1, 0},
    {"L1 qkv 256->768", 8, 32, 32, 256, 0, 768, 1, 1, 0},
    {"C4 384^2 conv 128->128", 1, 384, 384, 128, 0, 128, 3, 1, 0},
    {"C4 384^2 conv 256->128", 1, 384, 384, 256, 0, 128, 3, 1, 0},
    {"C4 384^2 conv 128->256", 1, 384, 384, 128, 0, 256, 3, 1, 0},
    {"C4 384^2 up 128 (192->384)", 1, 192, 192, 128, 0, 128, 3, 1, 1},
    {"C4 192^2 conv 128->128", 1, 192, 192, 128, 0, 128, 3, 1, 0},
    {"C4 192^2 conv 256->128", 1, 192, 192, 256, 0, 128, 3, 1, 0},
    {"C4 96^2 conv 256->256", 1, 96, 96, 256, 0, 256, 3, 1, 0},
    {"C4 96^2 conv 512->256", 1, 96, 96, 512, 0, 256, 3, 1, 0},
    {"C4 48^2 conv 256->256", 1, 48, 48, 256, 0, 256, 3, 1, 0},
    {"C4 48^2 conv 512->256", 1, 48, 48, 512, 0, 256, 3, 1, 0},
};

static uint16_t f2h(float v) {
    _Float16 h = (_Float16)v;
    uint16_t u;
    memcpy(&u, &h, 2);
    return u;
}
static float h2f(uint16_t u) {
    _Float16 h;
    memcpy(&h, &u, 2);
    return (float)h;
}

static int bench_main(int argc, char** argv);
int main(int argc, char** argv) {
    try {
        return bench_main(argc, argv);
    } catch (const cfd::Error& e) {
        fprintf(stderr, "cfd::Error %d: %s\n", e.code, e.msg.c_str());
        return 2;
    }
}

static int bench_main(int argc, char** argv) {
    std::vector<int> variants;
    for (int i = 1; i < argc; ++i) variants.push_back(atoi(argv[i]));
    if (variants.empty()) variants = {1, 2, 20};   // the K1x and K1h variants the planner ships (round 3)
    const int splits_x = getenv("CX_SPLITS") ? atoi(getenv("CX_SPLITS")) : 0;   // 0: auto
    hipStream_t st;
    CK(hipStreamCreate(&st));
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    const char* filt = getenv("CX_SHAPES");   // only shapes whose name contains this
    for (const Shape& s : SHAPES) {
        if (filt && !strstr(s.name, filt)) continue;
        const int Ctot = s.C1 + s.C2;
        const int Hout = s.up ? 2 * s.Hin : s.Hin / s.stride, Wout = s.up ? 2 * s.Win : s.Win / s.stride;
        const int M = s.B * Hout * Wout, K = s.ks * s.ks * Ctot;
        const size_t n1 = (size_t)s.B * s.Hin * s.Win * s.C1, n2 = (size_t)s.B * s.Hin * s.Win * s.C2;
        std::vector<float> x1(n1), x2(std::max<size_t>(n2, 1)), w((size_t)s.Cout * K), bias(s.Cout);
        for (auto& v : x1) v = U(rng);
        for (auto& v : x2) v = U(rng);
        const float wb = 1.f / std::sqrt((float)K);
        float amax = 0.f;
        for (auto& v : w) {
            v = U(rng) * wb;
            amax = std::max(amax, std::fabs(v));
        }
        for (auto& v : bias) v = U(rng) * wb;
        int ex = 0;
        std::frexp(amax, &ex);
        const float sc = std::ldexp(1.f, -ex);
        std::vector<uint16_t> wh(w.size()), wl(w.size());
        for (size_t e = 0; e < w.size(); ++e) {
            const float v = w[e] * sc;
            wh[e] = f2h(v);
            wl[e] = f2h(v - h2f(wh[e]));
        }
        float *d1, *d2, *dw, *db, *out0, *out1, *part;
        uint16_t *dh, *dl;
        CK(hipMalloc(&d1, n1 * 4));
        CK(hipMalloc(&d2, std::max<size_t>(n2, 1) * 4));
        CK(hipMalloc(&dw, w.size() * 4));
        CK(hipMalloc(&db, s.Cout * 4));
        CK(hipMalloc(&dh, w.size() * 2));
        CK(hipMalloc(&dl, w.size() * 2));
        CK(hipMalloc(&out0, (size_t)M * s.Cout * 4));
        CK(hipMalloc(&out1, (size_t)M * s.Cout * 4));
        const size_t part_floats = (size_t)16 * M * s.Cout;
        CK(hipMalloc(&part, part_floats * 4));
        CK(hipMemcpy(d1, x1.data(), n1 * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(d2, x2.data(), x2.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(db, bias.data(), s.Cout * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(dh, wh.data(), w.size() * 2, hipMemcpyHostToDevice));
        CK(hipMemcpy(dl, wl.data(), w.size() * 2, hipMemcpyHostToDevice));
        cfd::ConvArgs a{};
        a.src1 = d1;
        a.src2 = s.C2 ? d2 : nullptr;
        a.w = dw;
        a.wbf = dh;
        a.wlo = dl;
        a.acc_scale = 1.f / sc;
        a.bias = db;
        a.out = out0;
        a.part = part;
        a.C1 = s.C1;
        a.C2 = s.C2;
        a.Ctot = Ctot;
        a.Hin = s.Hin;
        a.Win = s.Win;
        a.Hout = Hout;
        a.Wout = Wout;
        a.stride = s.stride;
        a.ks = s.ks;
        a.pad = s.ks / 2;
        a.up = s.up;
        a.Cout = s.Cout;
        a.M = M;
        a.K = K;
        const double flops = 2.0 * M * s.Cout * K;
        const int iters = 20;
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        // reference: shipped planner + K1s (reduction included)
        const cfd::ConvPlan p = cfd::plan_conv(a, part_floats / 2);
        auto ref = [&]() { cfd::launch_conv(a, p, st, false); };
        ref();
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < iters; ++i) ref();
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms0;
        CK(hipEventElapsedTime(&ms0, e0, e1));
        ms0 /= iters;
        std::vector<float> r0((size_t)M * s.Cout), r1((size_t)M * s.Cout);
        CK(hipMemcpy(r0.data(), out0, r0.size() * 4, hipMemcpyDeviceToHost));
        float rmax = 0.f;
        for (float v : r0) rmax = std::max(rmax, std::fabs(v));
        printf("%-26s M=%6d N=%4d K=%5d | K1s %3dx%3d/%d split %2d: %8.1f us %6.1f TF\n", s.name, M, s.Cout, K, p.bm,
               p.bn, p.nw, p.splits, ms0 * 1e3, flops / (ms0 * 1e-3) / 1e12);
        for (int v : variants) {
            const int BMv_[] = {128, 128, 256, 128, 64, 64, 64, 128, 64, 128}, BNv_[] = {128, 128, 128, 64, 128, 64, 64, 64, 128, 128};
            const int vb = v >= 10 ? 0 : v;
            if (v == 30 && !splits_x) continue;
            const int BMv = v == 21 ? 128 : v >= 20 ? 256 : BMv_[vb], BNv = BNv_[vb];
            if ((v == 20 || v == 21) && !cfd::conv_h_tw(a)) continue;
            const int64_t tiles = ((M + BMv - 1) / BMv) * ((s.Cout + BNv - 1) / BNv);
            int splits = splits_x;
            if (!splits) {
                splits = 1;
                if (v == 20 || v == 21)
                    while (tiles * splits < 256 && Ctot / 32 / (splits * 2) >= (v == 21 ? 4 : 2) && splits < 16) splits *= 2;
                else
                    while (tiles * splits < 256 && K / 32 / (splits * 2) >= 8 && splits < 16) splits *= 2;
            }
            cfd::ConvArgs b = a;
            b.out = out1;
            b.xcd = 1;
            // variant 30: the shipped K1s tiles of the planner's choice at CX_SPLITS splits
            cfd::ConvPlan p30 = p;
            p30.splits = splits;
            p30.kx = -1;
            if (v == 30 && p30.bm == 256) p30.bm = 128;
            auto run = [&]() {
                if (v == 30) {
                    cfd::launch_conv(b, p30, st, false);
                    return;
                }
                cfd::launch_conv_x(b, v, splits, st);
                if (splits > 1) cfd::launch_splitk_reduce(b, splits, st);
            };
            CK(hipMemset(out1, 0, r1.size() * 4));
            run();
            CK(hipStreamSynchronize(st));
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < iters; ++i) run();
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms1;
            CK(hipEventElapsedTime(&ms1, e0, e1));
            ms1 /= iters;
            CK(hipMemcpy(r1.data(), out1, r1.size() * 4, hipMemcpyDeviceToHost));
            double dmax = 0;
            for (size_t e = 0; e < r1.size(); ++e) dmax = std::max(dmax, (double)std::fabs(r1[e] - r0[e]));
            printf("%-26s   variant %d split %2d: %8.1f us %6.1f TF  x%.2f  rel diff %.2e\n", "", v, splits,
                   ms1 * 1e3, flops / (ms1 * 1e-3) / 1e12, ms0 / ms1, dmax / rmax);
        }
        fflush(stdout);
        CK(hipFree(d1));
        CK(hipFree(d2));
        CK(hipFree(dw));
        CK(hipFree(db));
        CK(hipFree(dh));
        CK(hipFree(dl));
        CK(hipFree(out0));
        CK(hipFree(out1));
        CK(hipFree(part));
    }
    return 0;
}
