// Diffusion sampler epilogue (K6), Philox normals and latent de-normalisation.
//
// cfd_sched_step replaces, for ModelMeanType.EPSILON + ModelVarType.FIXED_LARGE,
//   _predict_xstart_from_eps -> clamp(-1,1) -> q_posterior_mean_variance
//   -> sample = mean + nonzero_mask * exp(0.5*logvar) * noise
// (U/src/gaussian_diffusion.py:300-314,328-333,208-230,395-439) and the DDIM
// update (:537-585).  Coefficients are the reference's float64 tables cast to
// fp32 per timestep (cast done once on the host, _extract_into_tensor :899-912);
// the elementwise maths is evaluated in the reference's operation order with
// fp contraction disabled, so for identical (x, eps, noise) the result is the
// reference's bit for bit.
#include <cmath>
#include <string>

#include "common.hpp"
#include "sampler.hpp"

namespace cfd {

struct Philox {
    static __device__ __forceinline__ uint4 round(uint4 c, uint2 k) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
        return make_uint4((uint32_t)(p1 >> 32) ^ c.y ^ k.x, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k.y,
                          (uint32_t)p0);
    }
    static __device__ __forceinline__ uint4 gen(uint64_t seed, uint64_t ctr_lo, uint64_t ctr_hi) {
        uint4 c = make_uint4((uint32_t)ctr_lo, (uint32_t)(ctr_lo >> 32), (uint32_t)ctr_hi, (uint32_t)(ctr_hi >> 32));
        uint2 k = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            c = round(c, k);
            k.x += 0x9E3779B9u;
            k.y += 0xBB67AE85u;
        }
        return c;
    }
    // Four N(0,1) floats for group `grp` of stream (seed, counter).
    static __device__ __forceinline__ void normal4(uint64_t seed, uint64_t counter, uint64_t grp, float z[4]) {
        const uint4 r = gen(seed, grp, counter);
        const float u1 = ((float)r.x + 1.0f) * 2.3283064365386963e-10f;  // (0, 1]
        const float u2 = (float)r.y * 2.3283064365386963e-10f;
        const float u3 = ((float)r.z + 1.0f) * 2.3283064365386963e-10f;
        const float u4 = (float)r.w * 2.3283064365386963e-10f;
        const float r1 = sqrtf(-2.0f * logf(fminf(u1, 1.0f)));
        const float r2 = sqrtf(-2.0f * logf(fminf(u3, 1.0f)));
        float s1, c1, s2, c2;
        sincospif(2.0f * u2, &s1, &c1);
        sincospif(2.0f * u4, &s2, &c2);
        z[0] = r1 * c1;
        z[1] = r1 * s1;
        z[2] = r2 * c2;
        z[3] = r2 * s2;
    }
};

__global__ void randn_kernel(float* __restrict__ out, int64_t n, uint64_t seed, uint64_t counter, uint64_t goff) {
    const int64_t grp = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t base = grp * 4;
    if (base >= n) return;
    float z[4];
    Philox::normal4(seed, counter, goff + (uint64_t)grp, z);
    if (base + 3 < n) {
        *(f4*)(out + base) = f4{z[0], z[1], z[2], z[3]};  // out 16-B aligned when n % 4 == 0 (checked by caller)
    } else {
        for (int j = 0; j < 4 && base + j < n; ++j) out[base + j] = z[j];
    }
}

struct StepArgs {
    const float* coefs;  // (n_t, CFD_NCOEF)
    const float* x;
    const float* eps;
    const int64_t* t;
    const float* noise;  // may be null -> Philox
    float* x_out;
    float* xs_out;       // may be null
    int64_t n;           // elements per sample
    int64_t total;       // B * n
    uint64_t seed, counter, goff;  // goff: Philox group offset (= element offset / 4)
    int kind, clip;
    const SamplerCtl* ctl;         // native loop: (seed, counter, goff) from device memory, or null
};

__global__ void step_kernel(StepArgs a) {
#pragma clang fp contract(off)
    const int64_t grp = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t base = grp * 4;
    if (base >= a.total) return;
    float z[4];
    if (a.noise) {
#pragma unroll
        for (int j = 0; j < 4; ++j) z[j] = (base + j < a.total) ? a.noise[base + j] : 0.f;
    } else if (a.ctl) {
        Philox::normal4(a.ctl->seed, a.ctl->counter, a.ctl->goff + (uint64_t)grp, z);
    } else {
        Philox::normal4(a.seed, a.counter, a.goff + (uint64_t)grp, z);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t i = base + j;
        if (i >= a.total) break;
        const int64_t b = i / a.n;
        const int64_t t = a.t[b];
        const float* c = a.coefs + t * CFD_NCOEF;
        const float x = a.x[i], e = a.eps[i];
        // pred_xstart = sqrt_recip_ac * x - sqrt_recipm1_ac * eps   (:328-333)
        float xs = c[CFD_COEF_SRA] * x - c[CFD_COEF_SRM1] * e;
        if (a.clip) xs = fminf(fmaxf(xs, -1.0f), 1.0f);
        const float mask = t != 0 ? 1.0f : 0.0f;
        float out;
        if (a.kind == CFD_STEP_DDPM) {
            // mean = coef1 * x0 + coef2 * x_t   (:217-220); sample (:431-438)
            const float mean = c[CFD_COEF_M1] * xs + c[CFD_COEF_M2] * x;
            out = mean + mask * c[CFD_COEF_SIGMA] * z[j];
        } else {
            // eps' = (sra * x - x0) / srm1 (:345-349); mean_pred (:566-570)
            const float e2 = (c[CFD_COEF_SRA] * x - xs) / c[CFD_COEF_SRM1];
            const float mean = xs * c[CFD_COEF_SQRT_ABP] + c[CFD_COEF_DIR] * e2;
            out = mean + mask * c[CFD_COEF_SIGMA_DDIM] * z[j];
        }
        a.x_out[i] = out;
        if (a.xs_out) a.xs_out[i] = xs;
    }
}

__global__ void latent_denorm_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n,
                                     const float* __restrict__ vmax, const float* __restrict__ vmin, int64_t period) {
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t k = i % period;
    // (gen + 1) * (max - min) / 2. + min   (scripts/inference.py:61)
    y[i] = (x[i] + 1.0f) * (vmax[k] - vmin[k]) / 2.0f + vmin[k];
}

// ---------------------------------------------------------------------------
// DPS glue: the elementwise links of
// d||y - A(x0_hat)|| / d x_t that are not the U-Net or SIREN adjoints.
// ---------------------------------------------------------------------------
// per sample b: r = y - A, norm_b = ||r||_2 (float64 sum), g_A = -r / norm_b
// (torch.linalg.norm backward; zero gradient where the norm is 0), condition_methods.py:33-35
__global__ __launch_bounds__(256) void dps_residual_kernel(const float* __restrict__ y, int64_t y_bstride,
                                                           const float* __restrict__ A, float* __restrict__ gA,
                                                           float* __restrict__ norm, int64_t n) {
    const int64_t b = blockIdx.x;
    const float* yb = y + b * y_bstride;
    const float* Ab = A + b * n;
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        const float r = yb[i] - Ab[i];
        s += (double)r * r;
    }
    __shared__ double red[256];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    const float nb = (float)sqrt(red[0]);
    if (threadIdx.x == 0) norm[b] = nb;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        const float r = yb[i] - Ab[i];
        gA[b * n + i] = nb > 0.f ? -(r / nb) : 0.f;
    }
}

// g_z -> (d_eps, g_direct) through Case4Operator._unnorm (measurements.py:219-220),
// clamp(-1, 1) (posterior_mean_variance.py:40-45; gradient passes on the closed
// interval) and x0 = sra * x - srm1 * eps (:120-123)
__global__ void dps_latent_grad_kernel(const float* __restrict__ coefs, int clip, const float* __restrict__ x,
                                       const float* __restrict__ eps, const int64_t* __restrict__ t,
                                       const float* __restrict__ gz, const float* __restrict__ vmax,
                                       const float* __restrict__ vmin, int64_t period, float* __restrict__ d_eps,
                                       float* __restrict__ g_direct, int64_t n, int64_t total) {
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int64_t b = i / n, k = i % period;
    const float* c = coefs + t[b] * CFD_NCOEF;
    const float x0u = c[CFD_COEF_SRA] * x[i] - c[CFD_COEF_SRM1] * eps[i];
    const bool pass = !clip || (x0u >= -1.0f && x0u <= 1.0f);
    const float gx0 = (gz[i] / 2.0f) * (vmax[k] - vmin[k]);
    const float g = pass ? gx0 : 0.0f;
    d_eps[i] = -g * c[CFD_COEF_SRM1];
    g_direct[i] = g * c[CFD_COEF_SRA];
}

// x_t -= (d/dx_prev) * scale   (condition_methods.py:88)
__global__ void dps_update_kernel(const float* __restrict__ sample, const float* __restrict__ g_direct,
                                  const float* __restrict__ g_unet, float scale, float* __restrict__ x_out,
                                  int64_t n) {
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    x_out[i] = sample[i] - (g_direct[i] + g_unet[i]) * scale;
}

// native loop bookkeeping (one workgroup): the step's timesteps from the
// host-built sequences, and the step counter for the Philox stream
__global__ void sampler_advance_kernel(SamplerCtl* ctl, const int64_t* __restrict__ tidx_seq,
                                       const int64_t* __restrict__ tmodel_seq, int64_t* __restrict__ t_idx,
                                       int64_t* __restrict__ t_model, int B) {
    const uint64_t k = ctl->k;
    for (int b = threadIdx.x; b < B; b += blockDim.x) {
        t_idx[b] = tidx_seq[k];
        t_model[b] = tmodel_seq[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        ctl->counter = k;
        ctl->k = k + 1;
    }
}

__global__ void sampler_set_kernel(SamplerCtl* ctl, uint64_t k, uint64_t seed, uint64_t goff) {
    if (threadIdx.x == 0) {
        ctl->k = k;
        ctl->counter = k;
        ctl->seed = seed;
        ctl->goff = goff;
    }
}

}  // namespace cfd

struct cfd_sched {
    float* coefs = nullptr;
    int n_t = 0;
    int device = 0;
};

namespace cfd {
const float* sched_coefs(const cfd_sched* s) { return s->coefs; }
int sched_nt(const cfd_sched* s) { return s->n_t; }

void launch_sampler_advance(SamplerCtl* ctl, const int64_t* tidx_seq, const int64_t* tmodel_seq, int64_t* t_idx,
                            int64_t* t_model, int B, hipStream_t st) {
    hipLaunchKernelGGL(sampler_advance_kernel, dim3(1), dim3(64), 0, st, ctl, tidx_seq, tmodel_seq, t_idx, t_model, B);
    check_launch("sampler_advance_kernel");
}

void launch_sampler_set(SamplerCtl* ctl, uint64_t k, uint64_t seed, uint64_t goff, hipStream_t st) {
    hipLaunchKernelGGL(sampler_set_kernel, dim3(1), dim3(64), 0, st, ctl, k, seed, goff);
    check_launch("sampler_set_kernel");
}

void launch_sched_step_ctl(const cfd_sched* s, int kind, int clip, float* x, const float* eps, const int64_t* t,
                           const SamplerCtl* ctl, int64_t n_per_sample, int B, hipStream_t st) {
    StepArgs a{s->coefs, x, eps, t, nullptr, x, nullptr, n_per_sample, n_per_sample * B, 0, 0, 0, kind, clip, ctl};
    const int64_t groups = ceil_div(a.total, 4);
    hipLaunchKernelGGL(step_kernel, dim3((unsigned)ceil_div(groups, 256)), dim3(256), 0, st, a);
    check_launch("step_kernel");
}
}  // namespace cfd

extern "C" int cfd_sched_create(const float* host_coefs, int n_t, int device, cfd_sched** out) {
    return cfd::guard([&] {
        CFD_REQUIRE(host_coefs && out && n_t > 0, CFD_EARG, "bad argument");
        cfd::DeviceGuard dg(device);
        auto* s = new cfd_sched();
        s->n_t = n_t;
        s->device = device;
        CFD_HIP(hipMalloc(&s->coefs, sizeof(float) * n_t * CFD_NCOEF));
        CFD_HIP(hipMemcpy(s->coefs, host_coefs, sizeof(float) * n_t * CFD_NCOEF, hipMemcpyHostToDevice));
        *out = s;
    });
}

extern "C" void cfd_sched_destroy(cfd_sched* s) {
    if (!s) return;
    (void)hipFree(s->coefs);
    delete s;
}

extern "C" int cfd_sched_step(const cfd_sched* s, int kind, int clip, const float* x, const float* eps,
                              const int64_t* t, const float* noise, uint64_t seed, uint64_t counter, uint64_t offset,
                              float* x_out, float* xstart_out, int64_t n_per_sample, int B, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(s && x && eps && t && x_out, CFD_EARG, "null argument");
        CFD_REQUIRE(offset % 4 == 0, CFD_EARG, "noise offset must be a multiple of 4");
        CFD_REQUIRE(kind == CFD_STEP_DDPM || kind == CFD_STEP_DDIM, CFD_EARG, "unknown step kind");
        CFD_REQUIRE(n_per_sample > 0 && B > 0, CFD_EARG, "empty step");
        cfd::StepArgs a{s->coefs, x, eps, t, noise, x_out, xstart_out, n_per_sample, n_per_sample * B,
                        seed, counter, offset / 4, kind, clip, nullptr};
        const int64_t groups = cfd::ceil_div(a.total, 4);
        hipLaunchKernelGGL(cfd::step_kernel, dim3((unsigned)cfd::ceil_div(groups, 256)), dim3(256), 0,
                           (hipStream_t)stream, a);
        cfd::check_launch("step_kernel");
    });
}

extern "C" int cfd_randn(float* out, int64_t n, uint64_t seed, uint64_t counter, uint64_t offset, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(out && n > 0, CFD_EARG, "bad argument");
        CFD_REQUIRE(offset % 4 == 0, CFD_EARG, "noise offset must be a multiple of 4");
        CFD_REQUIRE(((uintptr_t)out & 15) == 0, CFD_EARG, "randn output must be 16-byte aligned");
        const int64_t groups = cfd::ceil_div(n, 4);
        hipLaunchKernelGGL(cfd::randn_kernel, dim3((unsigned)cfd::ceil_div(groups, 256)), dim3(256), 0,
                           (hipStream_t)stream, out, n, seed, counter, offset / 4);
        cfd::check_launch("randn_kernel");
    });
}

extern "C" int cfd_latent_denorm(const float* x, float* y, int64_t n, const float* vmax, const float* vmin,
                                 int64_t period, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(x && y && vmax && vmin && n > 0 && period > 0, CFD_EARG, "bad argument");
        hipLaunchKernelGGL(cfd::latent_denorm_kernel, dim3((unsigned)cfd::ceil_div(n, 256)), dim3(256), 0,
                           (hipStream_t)stream, x, y, n, vmax, vmin, period);
        cfd::check_launch("latent_denorm_kernel");
    });
}

extern "C" int cfd_dps_residual(const float* y, int64_t y_batch_stride, const float* A, float* g_A, float* norm,
                                int64_t n_per_sample, int B, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(y && A && g_A && norm && n_per_sample > 0 && B > 0, CFD_EARG, "bad argument");
        CFD_REQUIRE(y_batch_stride == 0 || y_batch_stride == n_per_sample, CFD_EARG,
                    "measurement must be shared (stride 0) or per sample (stride n)");
        hipLaunchKernelGGL(cfd::dps_residual_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, y, y_batch_stride, A,
                           g_A, norm, n_per_sample);
        cfd::check_launch("dps_residual_kernel");
    });
}

extern "C" int cfd_dps_latent_grad(const cfd_sched* s, int clip, const float* x, const float* eps, const int64_t* t,
                                   const float* g_z, const float* vmax, const float* vmin, int64_t period,
                                   float* d_eps, float* g_direct, int64_t n_per_sample, int B, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(s && x && eps && t && g_z && vmax && vmin && d_eps && g_direct, CFD_EARG, "null argument");
        CFD_REQUIRE(n_per_sample > 0 && B > 0 && period > 0 && n_per_sample % period == 0, CFD_EARG,
                    "latent bounds must tile the latent");
        const int64_t total = n_per_sample * B;
        hipLaunchKernelGGL(cfd::dps_latent_grad_kernel, dim3((unsigned)cfd::ceil_div(total, 256)), dim3(256), 0,
                           (hipStream_t)stream, s->coefs, clip, x, eps, t, g_z, vmax, vmin, period, d_eps, g_direct,
                           n_per_sample, total);
        cfd::check_launch("dps_latent_grad_kernel");
    });
}

extern "C" int cfd_dps_update(const float* sample, const float* g_direct, const float* g_unet, float scale,
                              float* x_out, int64_t n, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(sample && g_direct && g_unet && x_out && n > 0, CFD_EARG, "bad argument");
        hipLaunchKernelGGL(cfd::dps_update_kernel, dim3((unsigned)cfd::ceil_div(n, 256)), dim3(256), 0,
                           (hipStream_t)stream, sample, g_direct, g_unet, scale, x_out, n);
        cfd::check_launch("dps_update_kernel");
    });
}

// ---------------------------------------------------------------------------
// Adam / AdamW (torch.optim.Adam / AdamW, fp32, amsgrad off; weight_decay > 0 is
// AdamW's decoupled decay, param *= 1 - lr wd, first): the optimisers of the CNF
// training loop (N/scripts/train.py:385-416) and of the diffusion TrainLoop (AdamW,
// U/src/train_util.py:78-80).  The reference steps them on its GPU, where torch's
// default is the multi-tensor (foreach) path of torch/optim/adam.py; per element,
// in that path's operation order and with the fused multiply-adds its device
// kernels execute (pinned bit for bit against torch.optim.AdamW on the MI355X by
// tests/test_gpu_optim.py; the probe is tools/dev/optim_probe.py):
//   exp_avg.lerp_(grad, 1 - beta1)          w < 0.5: fma(w, g - m, m)
//                                           else:    fma(-(g - m), 1 - w, g)
//   exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
//                                           fma(1 - beta2, g * g, v * beta2)
//   denom = exp_avg_sq.sqrt() / sqrt(1 - beta2^step) + eps   (IEEE sqrt, division)
//   param.addcdiv_(exp_avg, denom, value=-lr / (1 - beta1^step))
//                                           fma(-step_size, m / denom, p)
// The step-dependent scalars are formed in double on the host as torch does.
// torch's CPU kernels differ in two places (addcmul as fma(value * g, g, v),
// addcdiv as p + (value * m) / denom, and a vectorised sqrt that is not always
// correctly rounded): within an ulp of this on the same inputs.
// ---------------------------------------------------------------------------
namespace cfd {
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, int64_t n, float w1, float beta2, float w2, float bc2s, float eps,
                            float neg_step, float decay) {
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float pi = p[i];
    if (decay != 1.0f) pi = pi * decay;   // AdamW: param.mul_(1 - lr * weight_decay) first
    const float gi = g[i];
    float mi = m[i];
    mi = w1 < 0.5f ? __builtin_fmaf(w1, gi - mi, mi) : __builtin_fmaf(-(gi - mi), 1.0f - w1, gi);
    const float vi = __builtin_fmaf(w2, gi * gi, v[i] * beta2);
    const float denom = sqrtf(vi) / bc2s + eps;
    p[i] = __builtin_fmaf(neg_step, mi / denom, pi);
    m[i] = mi;
    v[i] = vi;
}
}  // namespace cfd

extern "C" int cfd_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, double lr,
                             double beta1, double beta2, double eps, double weight_decay, int64_t step, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(param && grad && exp_avg && exp_avg_sq && n >= 0 && step >= 1, CFD_EARG, "bad argument");
        CFD_REQUIRE(lr >= 0 && beta1 >= 0 && beta1 < 1 && beta2 >= 0 && beta2 < 1 && eps >= 0 && weight_decay >= 0,
                    CFD_EARG, "Adam hyper-parameters out of range");
        if (n == 0) return;
        const double bc1 = 1.0 - std::pow(beta1, (double)step), bc2 = 1.0 - std::pow(beta2, (double)step);
        const double step_size = lr / bc1, bc2s = std::sqrt(bc2);
        hipLaunchKernelGGL(cfd::adam_kernel, dim3((unsigned)cfd::ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream,
                           param, grad, exp_avg, exp_avg_sq, n, (float)(1.0 - beta1), (float)beta2,
                           (float)(1.0 - beta2), (float)bc2s, (float)eps, (float)(-step_size),
                           (float)(1.0 - lr * weight_decay));
        cfd::check_launch("adam_kernel");
    });
}
