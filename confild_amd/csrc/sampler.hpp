// Internal interface of the native reverse loop (sampler.hip): the pieces of
// unet.hip and diffusion.hip one captured sampler step is built from.
#pragma once
#include "common.hpp"

struct cfd_unet;
struct cfd_sched;

namespace cfd {

// Loop state the captured step reads from device memory instead of kernel
// arguments, so one instantiated graph serves every step of every loop.
struct SamplerCtl {
    uint64_t k;        // next step number (0 .. n_steps-1 in loop order)
    uint64_t counter;  // Philox counter of the step being run (= its step number, as the Python loop's k)
    uint64_t seed;     // Philox key of this loop
    uint64_t goff;     // Philox group offset (= element offset of the shard / 4)
};

// unet.hip: workspace size (cached per B) and the forward walk without the
// per-call checks (the sampler checks once at creation).
size_t unet_ws_bytes(const cfd_unet* h, int B);
void unet_check_ready(const cfd_unet* h);
int unet_compute(const cfd_unet* h);
uint64_t unet_version(const cfd_unet* h);
int unet_device(const cfd_unet* h);
int* unet_nonfinite(const cfd_unet* h);
void unet_forward_raw(const cfd_unet* h, const float* x, const int64_t* t, float* eps, int B, void* ws,
                      hipStream_t st);

// diffusion.hip
const float* sched_coefs(const cfd_sched* s);
int sched_nt(const cfd_sched* s);
// t_idx[b] = tidx_seq[k], t_model[b] = tmodel_seq[k], ctl->counter = k, ctl->k = k + 1
void launch_sampler_advance(SamplerCtl* ctl, const int64_t* tidx_seq, const int64_t* tmodel_seq, int64_t* t_idx,
                            int64_t* t_model, int B, hipStream_t st);
void launch_sampler_set(SamplerCtl* ctl, uint64_t k, uint64_t seed, uint64_t goff, hipStream_t st);
// cfd_sched_step with the Philox (seed, counter, offset) read from ctl, in place on x
void launch_sched_step_ctl(const cfd_sched* s, int kind, int clip, float* x, const float* eps, const int64_t* t,
                           const SamplerCtl* ctl, int64_t n_per_sample, int B, hipStream_t st);

}  // namespace cfd
