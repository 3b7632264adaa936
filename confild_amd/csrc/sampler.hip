// Native reverse loop: p_sample_loop / ddim_sample_loop (U/src/gaussian_diffusion.py:
// 441-535, 625-707) without per-step host work.
//
// The Python loop costs, per step, one ctypes U-Net call (~220 kernel launches,
// each a host-side dispatch) plus the timestep bookkeeping as torch ops -- at
// B = 1 the GPU waits on the host (config A: 2.6 ms per 19-GFLOP forward).  Here
// one step (timestep advance, U-Net forward, K6 epilogue in place) is captured
// once into a HIP graph; the step's timesteps and Philox counter live in device
// memory (SamplerCtl) and are advanced by the graph's first node, so the same
// instantiated graph replays every step of every loop.  `unroll` steps are
// captured back to back into one graph to amortise the graph launch.
//
// Results are bit-identical to the Python loop with Philox noise: the same
// kernels run with the same arguments; only the step's (seed, counter, offset)
// come from memory instead of kernel arguments.
#include <vector>

#include "sampler.hpp"

#include <hip/hip_ext.h>

struct cfd_sampler {
    const cfd_unet* unet = nullptr;
    const cfd_sched* sched = nullptr;
    int kind = 0, clip = 1, B = 0, n_steps = 0, device = 0, unroll = 1, graph = 1;
    int64_t n_per_sample = 0;
    float* x = nullptr;             // loop state (B, n_per_sample), updated in place
    float* eps = nullptr;
    int64_t* tseq = nullptr;        // (2, n_steps): table indices, then model timesteps
    int64_t* tbuf = nullptr;        // (2, B): this step's table index / model timestep per sample
    cfd::SamplerCtl* ctl = nullptr;
    void* ws = nullptr;             // U-Net workspace
    size_t ws_bytes = 0;            // (re-sized when the model's planned batch grows its split-K slab)
    // captured graphs: [0] one step, [1] `unroll` steps, and the U-Net handle version
    // they were captured at (a set_param can change a weight's split scale, which
    // is a kernel argument; set_compute changes the kernels)
    hipGraphExec_t exec[2] = {nullptr, nullptr};
    uint64_t exec_version = ~uint64_t(0);
};

namespace {

void destroy_graphs(cfd_sampler* sp) {
    for (auto& e : sp->exec)
        if (e) {
            (void)hipGraphExecDestroy(e);
            e = nullptr;
        }
    sp->exec_version = ~uint64_t(0);
}

// one reverse step on `st`: advance the timesteps, eps = U-Net(x, t), x = step(x, eps)
void enqueue_step(const cfd_sampler* sp, hipStream_t st) {
    cfd::launch_sampler_advance(sp->ctl, sp->tseq, sp->tseq + sp->n_steps, sp->tbuf, sp->tbuf + sp->B, sp->B, st);
    cfd::unet_forward_raw(sp->unet, sp->x, sp->tbuf + sp->B, sp->eps, sp->B, sp->ws, st);
    cfd::launch_sched_step_ctl(sp->sched, sp->kind, sp->clip, sp->x, sp->eps, sp->tbuf, sp->ctl, sp->n_per_sample,
                               sp->B, st);
}

hipGraphExec_t capture(const cfd_sampler* sp, int steps) {
    hipStream_t cs;
    CFD_HIP(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    hipGraph_t g = nullptr;
    hipGraphExec_t e = nullptr;
    try {
        CFD_HIP(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
        try {
            for (int i = 0; i < steps; ++i) enqueue_step(sp, cs);
        } catch (...) {
            hipGraph_t dummy = nullptr;
            (void)hipStreamEndCapture(cs, &dummy);
            if (dummy) (void)hipGraphDestroy(dummy);
            throw;
        }
        CFD_HIP(hipStreamEndCapture(cs, &g));
        CFD_HIP(hipGraphInstantiate(&e, g, nullptr, nullptr, 0));
    } catch (...) {
        if (g) (void)hipGraphDestroy(g);
        (void)hipStreamDestroy(cs);
        throw;
    }
    (void)hipGraphDestroy(g);
    (void)hipStreamDestroy(cs);
    return e;
}

}  // namespace

extern "C" int cfd_sampler_create(const cfd_unet* unet, const cfd_sched* sched, int kind, int clip, int B,
                                  int64_t n_per_sample, int n_steps, const int64_t* host_tidx,
                                  const int64_t* host_tmodel, int graph, int unroll, cfd_sampler** out) {
    return cfd::guard([&] {
        CFD_REQUIRE(unet && sched && out && host_tidx && host_tmodel, CFD_EARG, "null argument");
        CFD_REQUIRE(kind == CFD_STEP_DDPM || kind == CFD_STEP_DDIM, CFD_EARG, "unknown step kind");
        CFD_REQUIRE(B > 0 && n_steps > 0 && n_per_sample > 0, CFD_EARG, "empty loop");
        CFD_REQUIRE(unroll >= 1 && unroll <= 64, CFD_EARG, "unroll must be 1..64");
        cfd::unet_check_ready(unet);
        for (int k = 0; k < n_steps; ++k)
            CFD_REQUIRE(host_tidx[k] >= 0 && host_tidx[k] < cfd::sched_nt(sched), CFD_EARG,
                        "timestep index outside the coefficient table");
        cfd::DeviceGuard dg(cfd::unet_device(unet));
        auto* sp = new cfd_sampler();
        sp->unet = unet;
        sp->sched = sched;
        sp->kind = kind;
        sp->clip = clip ? 1 : 0;
        sp->B = B;
        sp->n_steps = n_steps;
        sp->n_per_sample = n_per_sample;
        sp->device = cfd::unet_device(unet);
        sp->graph = graph ? 1 : 0;
        sp->unroll = unroll;
        try {
            CFD_HIP(hipMalloc(&sp->x, sizeof(float) * (size_t)B * n_per_sample));
            CFD_HIP(hipMalloc(&sp->eps, sizeof(float) * (size_t)B * n_per_sample));
            CFD_HIP(hipMalloc(&sp->tseq, sizeof(int64_t) * 2 * (size_t)n_steps));
            CFD_HIP(hipMalloc(&sp->tbuf, sizeof(int64_t) * 2 * (size_t)B));
            CFD_HIP(hipMalloc(&sp->ctl, sizeof(cfd::SamplerCtl)));
            sp->ws_bytes = cfd::unet_ws_bytes(unet, B);
            CFD_HIP(hipMalloc(&sp->ws, sp->ws_bytes));
            CFD_HIP(hipMemcpy(sp->tseq, host_tidx, sizeof(int64_t) * n_steps, hipMemcpyHostToDevice));
            CFD_HIP(hipMemcpy(sp->tseq + n_steps, host_tmodel, sizeof(int64_t) * n_steps, hipMemcpyHostToDevice));
        } catch (...) {
            cfd_sampler_destroy(sp);
            throw;
        }
        *out = sp;
    });
}

extern "C" void cfd_sampler_destroy(cfd_sampler* sp) {
    if (!sp) return;
    destroy_graphs(sp);
    (void)hipFree(sp->x);
    (void)hipFree(sp->eps);
    (void)hipFree(sp->tseq);
    (void)hipFree(sp->tbuf);
    (void)hipFree(sp->ctl);
    (void)hipFree(sp->ws);
    delete sp;
}

extern "C" int cfd_sampler_run(cfd_sampler* sp, const float* x_in, float* x_out, int k0, int k1, uint64_t seed,
                               uint64_t offset, void* stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(sp, CFD_EARG, "null sampler");
        CFD_REQUIRE(0 <= k0 && k0 <= k1 && k1 <= sp->n_steps, CFD_EARG, "step range outside the loop");
        CFD_REQUIRE(offset % 4 == 0, CFD_EARG, "noise offset must be a multiple of 4");
        cfd::unet_check_ready(sp->unet);
        cfd::DeviceGuard dg(sp->device);
        const hipStream_t st = (hipStream_t)stream;
        if (const size_t need = cfd::unet_ws_bytes(sp->unet, sp->B); need > sp->ws_bytes) {
            // the model's planned batch changed (cfd_unet_set_plan_batch): a larger
            // slab, and graphs that captured the old workspace pointer are stale
            CFD_HIP(hipDeviceSynchronize());
            destroy_graphs(sp);
            CFD_HIP(hipFree(sp->ws));
            sp->ws = nullptr;
            sp->ws_bytes = 0;
            CFD_HIP(hipMalloc(&sp->ws, need));
            sp->ws_bytes = need;
        }
        const size_t bytes = sizeof(float) * (size_t)sp->B * sp->n_per_sample;
        if (x_in) CFD_HIP(hipMemcpyAsync(sp->x, x_in, bytes, hipMemcpyDeviceToDevice, st));
        cfd::launch_sampler_set(sp->ctl, (uint64_t)k0, seed, offset / 4, st);
        int k = k0;
        if (sp->graph) {
            if (sp->exec_version != cfd::unet_version(sp->unet)) {
                destroy_graphs(sp);
                sp->exec[0] = capture(sp, 1);
                if (sp->unroll > 1) sp->exec[1] = capture(sp, sp->unroll);
                sp->exec_version = cfd::unet_version(sp->unet);
            }
            for (; sp->unroll > 1 && k + sp->unroll <= k1; k += sp->unroll) CFD_HIP(hipGraphLaunch(sp->exec[1], st));
            for (; k < k1; ++k) CFD_HIP(hipGraphLaunch(sp->exec[0], st));
        } else {
            for (; k < k1; ++k) enqueue_step(sp, st);
        }
        if (x_out) CFD_HIP(hipMemcpyAsync(x_out, sp->x, bytes, hipMemcpyDeviceToDevice, st));
    });
}

extern "C" int cfd_device_cu_count(int device, int* n_cu) {
    return cfd::guard([&] {
        CFD_REQUIRE(n_cu, CFD_EARG, "null argument");
        hipDeviceProp_t p;
        CFD_HIP(hipGetDeviceProperties(&p, device));
        *n_cu = p.multiProcessorCount;
    });
}

extern "C" int cfd_stream_create_cu_range(int device, int first_cu, int n_cu, void** stream) {
    return cfd::guard([&] {
        CFD_REQUIRE(stream, CFD_EARG, "null argument");
        int total = 0;
        CFD_REQUIRE(cfd_device_cu_count(device, &total) == 0, CFD_EARG, "bad device");
        CFD_REQUIRE(first_cu >= 0 && n_cu > 0 && first_cu + n_cu <= total, CFD_EARG, "CU range outside the device");
        std::vector<uint32_t> mask((size_t)(total + 31) / 32, 0u);
        for (int c = first_cu; c < first_cu + n_cu; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
        cfd::DeviceGuard dg(device);
        hipStream_t s = nullptr;
        CFD_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
        *stream = (void*)s;
    });
}

extern "C" int cfd_stream_destroy(void* stream) {
    return cfd::guard([&] {
        if (stream) CFD_HIP(hipStreamDestroy((hipStream_t)stream));
    });
}
