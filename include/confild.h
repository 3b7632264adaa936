/*
 * confild.h -- C ABI of libconfild_hip.so, the MI355X (gfx950) implementation of
 * CoNFiLD's generation hot path.
 *
 * The reference (semihkacmaz/CoNFiLD, pure Python) has no native FFI: its
 * boundary is a set of Python callables.  Each entry point below replaces the
 * arithmetic behind one of them; the Python mirror in confild_amd/ binds these
 * with ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - plain pointers and sizes only; no framework types;
 *   - tensor pointers are DEVICE pointers on the handle's device unless the
 *     parameter name says host_; fp32 throughout (the reference computes fp32);
 *   - activations are NHWC ("channels last"); the U-Net's (B,1,H,W) input and
 *     output are identical in NCHW and NHWC because C == 1;
 *   - every call is stream-ordered on `stream` (a hipStream_t, NULL = default)
 *     and performs no host synchronisation, no allocation and no host<->device
 *     copy, except the *_create / *_set_param / cfd_sched_create calls;
 *   - return 0 on success, a CFD_E* code otherwise; cfd_last_error() gives a
 *     thread-local message.
 */
#ifndef CONFILD_H
#define CONFILD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { CFD_OK = 0, CFD_EARG = 1, CFD_EHIP = 2, CFD_EKEY = 3, CFD_ESHAPE = 4, CFD_ESTATE = 5 };

const char* cfd_last_error(void);
/* Returns the library build tag ("gfx950 ..."); used to prove which .so is loaded. */
const char* cfd_version(void);

/* ------------------------------------------------------------------------ */
/* Latent U-Net (replaces UNetModel, U/src/unet.py:396-663, built by         */
/* create_model, U/src/script_util.py:130-187).                              */
/* ------------------------------------------------------------------------ */
typedef struct cfd_unet cfd_unet;

typedef struct {
    int image_size;          /* informational; H == W == image_size expected   */
    int in_channels;         /* 1 in every CoNFiLD recipe                      */
    int model_channels;      /* num_channels                                   */
    int out_channels;        /* 1 (learn_sigma=False)                          */
    int num_res_blocks;
    int n_mult;              /* len(channel_mult)                              */
    int channel_mult[8];
    int n_attn;              /* len(attention downsample rates)                */
    int attention_ds[8];     /* image_size // res for res in attention_resolutions */
    int num_heads;
    int num_head_channels;   /* -1 => use num_heads                            */
} cfd_unet_cfg;

/* Builds the topology of UNetModel.__init__ (unet.py:427-616) on `device`. */
int  cfd_unet_create(const cfd_unet_cfg* cfg, int device, cfd_unet** out);
void cfd_unet_destroy(cfd_unet* h);
/* Parameter registry in the reference's state_dict order and key names. */
int  cfd_unet_num_params(const cfd_unet* h, int* n);
int  cfd_unet_param_info(const cfd_unet* h, int idx, const char** key, int* ndim, int64_t shape[4]);
/* Copies one reference-layout fp32 tensor (torch (Cout,Cin,kh,kw) etc.) from
 * HOST memory and packs it into the kernel layout.  Replaces load_state_dict. */
int  cfd_unet_set_param(cfd_unet* h, const char* key, const float* host_data, size_t n);
/* Overrides the (model_channels/2) timestep-embedding frequencies
 * exp(-ln(1e4) * i / half) (nn.py:129-131) with host-computed fp32 values so
 * they match the caller's framework bit for bit (default: computed in C++). */
int  cfd_unet_set_time_freqs(cfd_unet* h, const float* host_freqs, int n);
/* Fails with CFD_ESTATE until every parameter has been set. */
int  cfd_unet_ready(const cfd_unet* h);
/* Every parameter at once from a DEVICE buffer: `flat` holds the fp32 tensors
 * in cfd_unet_param_info order, reference layout, n floats in total.  Packs on
 * the device (the same layouts, bf16 copy, split-f16 hi / lo with the same
 * power-of-two scales as cfd_unet_set_param, bit for bit) on `stream` and
 * synchronises it once (the split scales are launch arguments).  The training
 * loop's parameter update (train_util.py: the optimizer writes the weights the
 * next forward reads).                                                         */
int  cfd_unet_load_flat(cfd_unet* h, const float* flat, size_t n, void* stream);
int  cfd_unet_workspace_bytes(const cfd_unet* h, int B, size_t* bytes);
/* eps = UNetModel.forward(x, timesteps): x (B,1,H,W), t (B) int64 (already
 * remapped through timestep_map, respace.py:123-128), eps (B,1,H,W). */
/* Convolution operand precision (config E, BASELINE.json configs[4]):
 * CFD_COMPUTE_BF16 rounds both convolution operands to bf16 (RNE) and
 * accumulates in fp32 on v_mfma_f32_16x16x32_bf16; GroupNorm, softmax, the
 * timestep MLP and the 1-channel in/out convolutions stay fp32, attention runs
 * the fp32-accurate split-f16 kernel.
 * Default CFD_COMPUTE_SPLIT_F16 (fp32-accurate, below); CFD_COMPUTE_F32 is the
 * exact fp32 MFMA path.  This
 * replaces UNetModel's use_fp16 torso conversion (U/src/unet.py:619-633) with
 * bf16 operands. */
/* CFD_COMPUTE_SPLIT_F16: fp32-accurate convolutions on f16 MFMA -- activations
 * and power-of-two-scaled weights split into f16 hi + lo (22-bit operands),
 * three v_mfma_f32_16x16x32_f16 per product (lo*hi + hi*lo + hi*hi), fp32
 * accumulation; error against an fp64 evaluation at the fp32 kernel's level
 * (DESIGN.md K1s).  Activations must stay below 65504 in magnitude. */
#define CFD_COMPUTE_F32       0
#define CFD_COMPUTE_BF16      1
#define CFD_COMPUTE_SPLIT_F16 2
int  cfd_unet_set_compute(cfd_unet* h, int compute);
/* The batch the convolution planner tiles for (tiles, split-K counts, kernel
 * family): 0 = 8 (default).  A per-model setting, never the real batch, so a
 * sample's eps stays bit-identical whatever batch or GPU it runs in; set it to
 * the chains a GPU runs when that is far from 8 (real Case4 at one chain: 2,
 * +8 % steps/s).  No reference counterpart (a performance setting). */
int  cfd_unet_set_plan_batch(cfd_unet* h, int nominal_batch);
int  cfd_unet_forward(cfd_unet* h, const float* x, const int64_t* t, float* eps, int B,
                      void* workspace, size_t ws_bytes, void* stream);
/* Range guard of the split-f16 compute (no reference counterpart: the
 * reference's fp32 aten ops have no f16 range).  Every forward's last
 * convolution raises a device flag when an eps value is not finite -- an
 * activation beyond 65504 makes its f16 hi part infinite and reaches eps as
 * inf / NaN.  Reads the flag accumulated since the previous call (stream-
 * ordered, synchronises `stream`) into *nonfinite and clears it. */
int  cfd_unet_check_finite(cfd_unet* h, int* nonfinite, void* stream);

/* Input-gradient of the U-Net (DPS adjoint; replaces the autograd.grad of
 * grad_and_value through UNetModel.forward, C/src/guided_diffusion/
 * condition_methods.py:31-47, C/unet.py).  cfd_unet_forward_tape is
 * cfd_unet_forward (bit-identical eps) that also keeps every activation the
 * backward needs in `tape`; cfd_unet_input_vjp then computes
 * d_x = (d eps / d x)^T d_eps for that forward (same h, B and tape).  Weights are
 * constants: no parameter gradients. */
int  cfd_unet_tape_bytes(const cfd_unet* h, int B, size_t* bytes);
int  cfd_unet_vjp_workspace_bytes(const cfd_unet* h, int B, size_t* bytes);
int  cfd_unet_forward_tape(cfd_unet* h, const float* x, const int64_t* t, float* eps, int B,
                           void* workspace, size_t ws_bytes, void* tape, size_t tape_bytes, void* stream);
int  cfd_unet_input_vjp(cfd_unet* h, const float* d_eps, float* d_x, int B, const void* tape,
                        size_t tape_bytes, void* workspace, size_t ws_bytes, void* stream);
/* What the next cfd_unet_forward_tape records (and cfd_unet_tape_bytes sizes):
 * CFD_TAPE_INPUT_VJP (default) the activations cfd_unet_input_vjp reads, nothing
 * more (the DPS adjoint); CFD_TAPE_PARAM_GRAD also every GroupNorm(+SiLU) output
 * the convolutions read and its max |.| -- the operands of cfd_unet_param_grad's
 * split weight gradients, which otherwise recompute them (one activation per
 * GroupNorm of tape memory, +0.3 ms per Case1 forward, -2.5 ms per backward).
 * The handle remembers, per tape pointer, the mode, batch and planned batch each
 * cfd_unet_forward_tape recorded (the 64 most recent tapes): input_vjp /
 * param_grad replay THAT tape's layout, so several live tapes of different modes
 * stay valid; replaying a tape the handle did not record (or recorded at another
 * B or plan) fails with CFD_ESTATE / CFD_EARG instead of reading a wrong layout. */
#define CFD_TAPE_INPUT_VJP  0
#define CFD_TAPE_PARAM_GRAD 1
int  cfd_unet_set_tape_mode(cfd_unet* h, int mode);

/* ------------------------------------------------------------------------ */
/* Diffusion step epilogue (replaces p_mean_variance + p_sample / ddim_sample */
/* for EPSILON / FIXED_LARGE, U/src/gaussian_diffusion.py:232-326,395-439,    */
/* 537-585).                                                                   */
/* ------------------------------------------------------------------------ */
typedef struct cfd_sched cfd_sched;
enum { CFD_COEF_SRA = 0, CFD_COEF_SRM1, CFD_COEF_M1, CFD_COEF_M2, CFD_COEF_SIGMA,
       CFD_COEF_SQRT_ABP, CFD_COEF_DIR, CFD_COEF_SIGMA_DDIM, CFD_NCOEF };
enum { CFD_STEP_DDPM = 0, CFD_STEP_DDIM = 1 };

/* host_coefs: n_t rows of CFD_NCOEF fp32 values, the float64 tables of the
 * (respaced) process already cast to fp32 the way _extract_into_tensor does
 * (gaussian_diffusion.py:899-912). */
int  cfd_sched_create(const float* host_coefs, int n_t, int device, cfd_sched** out);
void cfd_sched_destroy(cfd_sched* s);
/* x_out = step(x, eps, t).  t: (B) int64 device indices into the table.
 * noise: (B*n) device normals in the reference's draw order, or NULL to draw
 * them in-kernel with Philox4x32-10 keyed by (seed, counter); element i of
 * this call uses stream position offset + i (offset % 4 == 0), so a batch
 * sharded over ranks draws exactly the normals of the unsharded batch.
 * xstart_out may be NULL.  x_out may alias x. */
int  cfd_sched_step(const cfd_sched* s, int kind, int clip, const float* x, const float* eps,
                    const int64_t* t, const float* noise, uint64_t seed, uint64_t counter,
                    uint64_t offset, float* x_out, float* xstart_out, int64_t n_per_sample, int B,
                    void* stream);
/* Native reverse loop (p_sample_loop / ddim_sample_loop, gaussian_diffusion.py:
 * 441-535 / 625-707, with Philox noise): per step the timestep advance, the U-Net
 * forward and the K6 epilogue, with no host work between steps.  graph != 0
 * captures the step once into a HIP graph (`unroll` steps per graph, 1..64) and
 * replays it; the step's timesteps and Philox counter live in device memory.
 * host_tidx[k] / host_tmodel[k]: coefficient-table index / model timestep
 * (timestep_map) of step k in loop order.  The sampler owns its state, eps and
 * U-Net workspace; `unet` and `sched` must outlive it.  Parameters set on
 * `unet` later and compute-mode changes are seen (the graph is re-captured
 * when the handle changed since the last capture).
 * cfd_sampler_run: steps [k0, k1) of the loop; x_in (B * n_per_sample) is
 * copied in first unless NULL (continue from the state), x_out receives the
 * state afterwards unless NULL.  Step k draws Philox(seed, counter = k) at
 * stream position offset + element (offset % 4 == 0), exactly as
 * cfd_sched_step with counter k, so the result is bit-identical to a host loop
 * of cfd_unet_forward + cfd_sched_step. */
typedef struct cfd_sampler cfd_sampler;
int  cfd_sampler_create(const cfd_unet* unet, const cfd_sched* sched, int kind, int clip, int B,
                        int64_t n_per_sample, int n_steps, const int64_t* host_tidx, const int64_t* host_tmodel,
                        int graph, int unroll, cfd_sampler** out);
void cfd_sampler_destroy(cfd_sampler* sp);
/* A stream whose kernels run on CUs [first_cu, first_cu + n_cu) of the device only
 * (hipExtStreamCreateWithCUMask): the sampling loop and the CNF decode of the
 * previous batch run side by side on disjoint halves of the chip (bench.py config
 * B).  No reference counterpart (an execution resource). */
int  cfd_device_cu_count(int device, int* n_cu);
int  cfd_stream_create_cu_range(int device, int first_cu, int n_cu, void** stream);
int  cfd_stream_destroy(void* stream);
int  cfd_sampler_run(cfd_sampler* sp, const float* x_in, float* x_out, int k0, int k1, uint64_t seed,
                     uint64_t offset, void* stream);
/* n standard normals from Philox4x32-10 (seed, counter) at stream positions
 * offset .. offset+n-1 (offset % 4 == 0): the device-side stand-in for th.randn
 * (gaussian_diffusion.py:513). */
int  cfd_randn(float* out, int64_t n, uint64_t seed, uint64_t counter, uint64_t offset, void* stream);
/* Diagnostic: y = sin(x) by the decoder's device sine -- which 0: Cody-Waite pi
 * reduction + degree-9 polynomial (sin_cw family), 1: Cody-Waite 2pi reduction +
 * v_sin_f32, 2: reduction in revolutions (two-float 1/2pi) + v_sin_f32 (the
 * split32 decoder's default).  Used by the tests to bound each against float64
 * (components.py:19-25 Sine = torch.sin). */
int  cfd_sine_probe(const float* x, float* y, int64_t n, int which, void* stream);
/* Latent de-normalisation (scripts/inference.py:59-61): y = (x+1)*(max-min)/2 + min,
 * max/min broadcast over the trailing `period` elements (period=1: scalars). */
int  cfd_latent_denorm(const float* x, float* y, int64_t n, const float* vmax, const float* vmin,
                       int64_t period, void* stream);

/* DPS glue (Case4 conditional sampling, C/src/guided_diffusion/condition_methods.py:31-47,81-90):
 *   cfd_dps_residual     per sample: norm_b = ||y - A_b||_2, g_A = -(y - A_b) / norm_b
 *                        (y shared when y_batch_stride == 0, else per sample);
 *   cfd_dps_latent_grad  g_z (d norm / d unnormalised latent) -> d_eps = -srm1 * g and
 *                        g_direct = sra * g, g = clamp'(x0) * g_z * (max - min) / 2
 *                        (Case4Operator._unnorm, measurements.py:219-220);
 *   cfd_dps_update       x_out = sample - (g_direct + g_unet) * scale. */
int  cfd_dps_residual(const float* y, int64_t y_batch_stride, const float* A, float* g_A, float* norm,
                      int64_t n_per_sample, int B, void* stream);
int  cfd_dps_latent_grad(const cfd_sched* s, int clip, const float* x, const float* eps, const int64_t* t,
                         const float* g_z, const float* vmax, const float* vmin, int64_t period,
                         float* d_eps, float* g_direct, int64_t n_per_sample, int B, void* stream);
int  cfd_dps_update(const float* sample, const float* g_direct, const float* g_unet, float scale,
                    float* x_out, int64_t n, void* stream);

/* ------------------------------------------------------------------------ */
/* Conditional neural field decoder: SIRENAutodecoder_film                    */
/* (N/cnf/nf_networks.py:443-495, BatchLinear/Sine components.py:19-25,55-76) */
/* fused with Normalizer_ts '-11' (N/cnf/utils/normalize.py:100-114).         */
/* ------------------------------------------------------------------------ */
typedef struct cfd_siren cfd_siren;

typedef struct {
    int in_coord_features;   /* d  (<= 4)                                     */
    int in_latent_features;  /* L                                            */
    int out_features;        /* c  (<= 4)                                     */
    int num_hidden_layers;   /* nh                                           */
    int hidden_features;     /* H  (multiple of 16, <= 512)                  */
    float w0;                /* 30 (DEFAULT_W0)                              */
} cfd_siren_cfg;

int  cfd_siren_create(const cfd_siren_cfg* cfg, int device, cfd_siren** out);
void cfd_siren_destroy(cfd_siren* h);
int  cfd_siren_num_params(const cfd_siren* h, int* n);
int  cfd_siren_param_info(const cfd_siren* h, int idx, const char** key, int* ndim, int64_t shape[4]);
/* keys net1.{i}.weight/bias, net2.{i}.weight (host fp32, reference layout). */
int  cfd_siren_set_param(cfd_siren* h, const char* key, const float* host_data, size_t n);
int  cfd_siren_ready(const cfd_siren* h);
int  cfd_siren_workspace_bytes(const cfd_siren* h, int b, size_t* bytes);
/* out (b, N, c) = denorm( NF( norm(coords), latents ) ).
 *   coords (N, d); latents (b, L);
 *   xmax/xmin: (d) coordinate normaliser params, or NULL (coords already normalised);
 *   ymax/ymin: output normaliser params with row stride y_stride (elements) per
 *              coordinate: y_stride = c for a per-point (N, c) table (lumped
 *              latent, train.py:194-201), 0 for a (c) table; NULL = raw output. */
/* Hidden-layer arithmetic of cfd_siren_forward:
 * CFD_SIREN_SPLIT_F16 (default; H a multiple of 32, nh >= 1): every product W x
 *   as three v_mfma_f32_16x16x32_f16 on two-term f16 splits of the power-of-two
 *   scaled weights and of the activations (Wl xh + Wh xl + Wh xh, fp32
 *   accumulate): 22-bit operands, exact products, fp32 accumulation -- the error
 *   against an fp64 evaluation matches the fp32 chain's;
 * CFD_SIREN_F32: the exact fp32 v_mfma_f32_16x16x4_f32 chain.
 * Env CFD_SIREN_COMPUTE overrides the default at handle creation.
 * cfd_siren_get_compute reports the mode a forward actually runs. */
#define CFD_SIREN_F32       0
#define CFD_SIREN_SPLIT_F16 1
int  cfd_siren_set_compute(cfd_siren* h, int compute);
int  cfd_siren_get_compute(const cfd_siren* h, int* compute);
int  cfd_siren_forward(cfd_siren* h, const float* coords, int64_t N, const float* latents, int b,
                       const float* xmax, const float* xmin,
                       const float* ymax, const float* ymin, int64_t y_stride,
                       float* out, void* workspace, size_t ws_bytes, void* stream);

/* Latent-gradient of the Case4 measurement operator (DPS; replaces autograd
 * through Case4Operator.forward -> pass_through_model_batch -> SIRENAutodecoder_film,
 * C/src/guided_diffusion/measurements.py:219-226, N/cnf/inference_function.py:22-48).
 * cfd_siren_tape_forward = cfd_siren_forward over Ns sensor coordinates for R
 * latent rows, keeping each layer's pre-activation in the workspace;
 * cfd_siren_tape_vjp: g_latents (R, L) = d<g_out, out>/d latents for that forward
 * (same h, Ns, R, workspace and y normaliser). */
int  cfd_siren_vjp_workspace_bytes(const cfd_siren* h, int64_t Ns, int R, size_t* bytes);
int  cfd_siren_tape_forward(cfd_siren* h, const float* coords, int64_t Ns, const float* latents, int R,
                            const float* xmax, const float* xmin,
                            const float* ymax, const float* ymin, int64_t y_stride,
                            float* out, void* workspace, size_t ws_bytes, void* stream);
int  cfd_siren_tape_vjp(cfd_siren* h, const float* g_out, int64_t Ns, int R,
                        const float* ymax, const float* ymin, int64_t y_stride,
                        float* g_latents, void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------ */
/* CNF autodecoder training (K10; N/scripts/train.py:334-416 _single_trainer:  */
/* model(coords, latents(idx)) -> MSELoss -> loss.backward(), Adam steps).     */
/* ------------------------------------------------------------------------ */
/* One backward of MSELoss(mean) for a batch: R latent rows (rows[r] indexes   *
 * the (N_samples, L) latent table `latents`, distinct), N raw coordinates     *
 * (N, d) as the model sees them, target (R, N, c).  scale = 2 / (numel of the *
 * whole loss) (ATen mse_loss_backward's factor; a caller that splits the      *
 * coordinates over several calls passes the full count).  Accumulates (+=):   *
 *   grad          flat fp32 gradient, parameters in cfd_siren_param_info order *
 *                 and reference shapes (torch's .grad accumulation);          *
 *   grad_latents  (N_samples, L): the batch's rows;                           *
 *   sse           (1) sum of squared errors of this call.                     *
 * fp32 throughout (fp32 MFMA tape chain, fp32 MFMA weight-gradient products   *
 * over the (row, coordinate) pairs); deterministic.                           */
int  cfd_siren_train_workspace_bytes(const cfd_siren* h, int64_t N, int R, size_t* bytes);
int  cfd_siren_train_grad(cfd_siren* h, const float* coords, int64_t N, const float* latents,
                          const int64_t* rows, int R, const float* target, float scale,
                          float* grad, float* grad_latents, float* sse,
                          void* workspace, size_t ws_bytes, void* stream);
/* ------------------------------------------------------------------------ */
/* Latent U-Net parameter gradients (K11; the diffusion TrainLoop's backward,  */
/* U/src/train_util.py:196-240 -> loss.backward() through UNetModel.forward).  */
/* ------------------------------------------------------------------------ */
/* For the forward recorded by cfd_unet_forward_tape(h, x, t, ...) on `tape`:   *
 * grad (flat fp32, cfd_unet_param_info order and reference shapes) +=         *
 * (d eps / d params)^T d_eps -- every convolution weight / bias, GroupNorm    *
 * gamma / beta, emb_layers and time_embed parameter; x is that forward's      *
 * input.  fp32 (fp32 MFMA weight-gradient products over the pixels, fixed     *
 * reduction orders: deterministic).                                           */
int  cfd_unet_param_grad_workspace_bytes(const cfd_unet* h, int B, size_t* bytes);
int  cfd_unet_param_grad(cfd_unet* h, const float* x, const float* d_eps, int B, const void* tape,
                         size_t tape_bytes, float* grad, void* workspace, size_t ws_bytes, void* stream);
/* GaussianDiffusion.training_losses' MSE term on eps (gaussian_diffusion.py    *
 * :775-853) and the backward of (loss * weights).mean() (train_util.py:210):   *
 * d_eps = scale * weights[b] * (eps - noise) (scale = 2 / numel for the batch  *
 * mean of mean_flat; weights may be null = 1), sse[b] = sum over sample b of   *
 * (eps - noise)^2.                                                             */
int  cfd_eps_mse(const float* eps, const float* noise, const float* weights, float* d_eps,
                 int64_t n_per_sample, int B, float scale, float* sse, void* stream);
/* update_ema (U/src/nn.py:71-80): target = target * rate + source * (1 - rate). */
int  cfd_ema_update(float* target, const float* source, int64_t n, double rate, void* stream);
/* q_sample (U/src/gaussian_diffusion.py:188-206): x_t = coef_a[b] x0 +        *
 * coef_s[b] noise per sample, coef_a / coef_s the fp32 casts of              *
 * sqrt(alphas_cumprod[t]) / sqrt(1 - alphas_cumprod[t]).                      */
int  cfd_q_sample(const float* x0, const float* noise, const float* coef_a, const float* coef_s, float* x_t,
                  int64_t n_per_sample, int B, void* stream);
/* torch.optim.Adam / AdamW step (amsgrad off) over n fp32 elements: exp_avg /  *
 * exp_avg_sq updated in place, step = the 1-based step count; weight_decay > 0 *
 * is AdamW's decoupled decay (param *= 1 - lr * weight_decay first).           */
int  cfd_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                   double lr, double beta1, double beta2, double eps, double weight_decay, int64_t step,
                   void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CONFILD_H */
