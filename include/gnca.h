/*
 * gnca.h — C ABI of the MI355X-native NCA rollout step (libgnca.so).
 *
 * This is the drop-in boundary for ONE hot path of Psylocibe23/Graph_Neural_Cellular_Automata:
 * the per-cell CA update of NeuralCAGraph.forward / NeuralCA.forward plus the mid-range graph
 * residual of GraphAugmentation.forward.  The reference has no FFI of its own: its boundary is
 * the Python nn.Module API, and the Python package graph_neural_cellular_automata_amd mirrors
 * that API on top of these entry points (ctypes).  INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - Every tensor pointer is DEVICE memory, fp32, NCHW contiguous (the reference's layout),
 *     caller-owned.  Weight pointers use the reference's parameter layouts (Conv2d weights
 *     [out,in,1,1] / [3C,1,3,3]); no host-side repacking is needed.
 *   - All work is stream-ordered on `stream`; no entry point synchronises the device, allocates
 *     memory or copies host<->device, so calls can be captured into a hipGraph.
 *   - Return value: 0 (GNCA_OK) or a negative gnca_status; gnca_status_string() names it.
 *   - Stateless and reentrant (gnca_rollout_f32's sub-batch streams are per-device helpers whose
 *     enqueue is serialised by an internal lock).
 *
 * Reference interfaces replaced (paths relative to the reference root):
 *   gnca_step_f32        NeuralCAGraph.forward        src/modules/ncagraph.py:106-168
 *                        NeuralCA.forward (graph off) src/modules/nca.py:64-105
 *                        GraphAugmentation.forward    src/modules/graph_augmentation.py:104-169
 *                        FixedSobelPerception.forward src/modules/perception.py:21-26
 *   gnca_message_f32     GraphAugmentation.forward    src/modules/graph_augmentation.py:104-169
 *   gnca_perceive_f32    FixedSobelPerception.forward src/modules/perception.py:21-26
 *   gnca_rollout_f32     the rollout loops that call the step once per CA step, e.g.
 *                        src/training/train_graph_augmented_nca.py:305-321,
 *                        src/testing/test_graph_augmented_regeneration.py:183-194
 *   gnca_damage_f32      the damage curriculum's batch ops, src/utils/damage.py:15-138
 *   gnca_step_bwd_f32    torch autograd's backward through NeuralCAGraph.forward /
 *                        NeuralCA.forward, i.e. the per-step part of the trainers'
 *                        loss.backward() (BPTT): src/training/train_graph_augmented_nca.py:369,
 *                        src/training/train_intermediate_loss.py (same loop)
 */
#ifndef GNCA_H
#define GNCA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GNCA_ABI_VERSION 2
#define GNCA_MAX_OFFSETS 128   /* >= (2r+1)^2-9 for r <= 5 (112) */

/* gnca_step_desc.flags */
#define GNCA_GRAPH          (1u << 0)  /* NeuralCAGraph (graph message on); clear = NeuralCA  */
#define GNCA_USE_GROUPNORM  (1u << 1)  /* nn.GroupNorm(1,C,eps) on dx (ncagraph.py:68)       */
#define GNCA_HIDDEN_ONLY    (1u << 2)  /* zero message channels 0..3 (ncagraph.py:98-100)     */
#define GNCA_ALIVE_TO_ALIVE (1u << 3)  /* mask messages by sender alive (graph_aug.py:131)   */
#define GNCA_ZERO_PAD_SHIFT (1u << 4)  /* _shift2d_pad (dx ignored) instead of torch.roll     */
#define GNCA_ATTENTION      (1u << 5)  /* also write the normalised attention map [B,H,W]    */

/* gnca_step_desc.fire_mode: the stochastic fire mask of ncagraph.py:144-146 */
#define GNCA_FIRE_NONE      0  /* fire_rate >= 1: no mask                                   */
#define GNCA_FIRE_RAND_F32  1  /* fire = (fire[b,0,i,j] <= fire_rate), fire = torch.rand(B,1,H,W) */
#define GNCA_FIRE_MASK_U8   2  /* fire = (fire[b,0,i,j] != 0), an explicit uint8 mask         */
#define GNCA_FIRE_HASH      3  /* counter RNG: u(seed, rng_step, sample_base+b, i*W+j) <= fire_rate */

typedef enum gnca_status {
  GNCA_OK = 0,
  GNCA_ERR_INVALID = -1,      /* bad shape / argument / null pointer                      */
  GNCA_ERR_UNSUPPORTED = -2,  /* shape class not compiled in (C > 32, hidden > 256, ...)  */
  GNCA_ERR_WORKSPACE = -3,    /* workspace too small (see gnca_workspace_bytes)            */
  GNCA_ERR_HIP = -4           /* a HIP launch failed; gnca_last_hip_error() has the code   */
} gnca_status;

typedef struct gnca_step_desc {
  int32_t B, C, H, W;         /* state shape, C >= 4 (alpha is channel 3)                    */
  int32_t hidden;             /* update_hidden (update_net.0 out channels)                   */
  int32_t d_model;            /* graph d_model (query/key channels)                          */
  int32_t num_offsets;        /* k = len(chosen offsets) this step, 0..GNCA_MAX_OFFSETS      */
  int32_t fire_mode;          /* GNCA_FIRE_*                                                 */
  uint32_t flags;             /* GNCA_* flag bits                                            */
  float update_gain;          /* NeuralCAGraph.update_gain                                    */
  float alpha_thr;            /* NeuralCAGraph.alpha_thr: pre/post-update alive masks         */
  float graph_alpha_thr;      /* GraphAugmentation.alpha_thr: sender mask (copied at ctor,
                                 ncagraph.py:79 -> graph_augmentation.py:52,117)              */
  float message_gain;         /* NeuralCAGraph.message_gain, read per call                    */
  float gn_eps;               /* GroupNorm eps (1e-3 in the reference)                        */
  float fire_rate;            /* forward(fire_rate)                                          */
  uint64_t rng_seed;          /* GNCA_FIRE_HASH only                                          */
  int64_t rng_step;           /* GNCA_FIRE_HASH only: step index in the rollout               */
  int64_t sample_base;        /* GNCA_FIRE_HASH only: global index of sample 0 of this shard  */
  int8_t offsets[2 * GNCA_MAX_OFFSETS]; /* (dy,dx) pairs in random.sample order            */
} gnca_step_desc;

typedef struct gnca_weights {
  const float* perception;    /* perception.conv.weight [3C,1,3,3]                          */
  const float* w1;            /* update_net.0.weight    [hidden,3C,1,1]                     */
  const float* b1;            /* update_net.0.bias      [hidden]                            */
  const float* w2;            /* update_net.2.weight    [C,hidden,1,1]                      */
  const float* gn_weight;     /* norm.weight [C] (NULL if !GNCA_USE_GROUPNORM)              */
  const float* gn_bias;       /* norm.bias   [C]                                            */
  const float* wq;            /* graph.query_proj.weight [d,C,1,1]  (graph only)            */
  const float* bq;            /* graph.query_proj.bias   [d]                                */
  const float* wk;            /* graph.key_proj.weight   [d,C,1,1]                          */
  const float* bk;            /* graph.key_proj.bias     [d]                                */
  const float* wm;            /* graph.msg_proj.weight   [C,C,1,1]                          */
  const float* bm;            /* graph.msg_proj.bias     [C]                                */
  const float* scaling;       /* graph.scaling           [] (device scalar)                 */
} gnca_weights;

/* ABI version (GNCA_ABI_VERSION) — lets a binding check it loaded a matching library. */
int gnca_abi_version(void);

/* Human-readable name of a gnca_status. */
const char* gnca_status_string(int status);

/* The hipError_t of the last failed launch on this thread (0 if none). */
int gnca_last_hip_error(void);

/* Bytes of device workspace gnca_step_f32 needs for `desc` (0 on invalid desc). */
size_t gnca_workspace_bytes(const gnca_step_desc* desc);

/* Measurement: the K1 kernel the plan for `desc` launches, as "name<template args>" (NUL-terminated,
 * truncated to n bytes), and its MFMA arithmetic in *arith (may be NULL): 0 = fp32 MFMA
 * (v_mfma_f32_*_f32), 1 = bf16 MFMA on exact 3-way splits of the fp32 operands (6 products per
 * fp32 product, gnca_k1_split.h), plus 2 when a rollout of this shape uses the compact update field
 * (GNCA_PHASE_COMPACT), plus 4 when a rollout of this shape runs as 2 concurrent sub-batches (one
 * stream each: one sub-batch's K2 beside the other's K1; see gnca_rollout_f32), plus 8 when a
 * rollout of this shape folds each step's finish (GroupNorm, tanh, residual, alpha gate) into the
 * next step's K1 (one K1 launch per step and one K2 at the end), plus 16 when such a fold is
 * possible for this shape (on request, GNCA_ROLLOUT_FOLD, where it is not the default).  Host-only.
 * Returns GNCA_OK or GNCA_ERR_INVALID. */
int gnca_k1_variant(const gnca_step_desc* desc, char* name, int32_t n, int32_t* arith);

/*
 * One CA step: x_out = step(x).  Out-of-place (x_out must not alias x), like the reference.
 *   fire:  NULL, or [B,1,H,W] fp32 uniforms (GNCA_FIRE_RAND_F32) / uint8 mask (GNCA_FIRE_MASK_U8)
 *   attn:  [B,H,W] fp32, written iff GNCA_ATTENTION (min-max normalised, graph_aug.py:160-167)
 *   ws:    >= gnca_workspace_bytes(desc) bytes of device memory, 256-B aligned
 */
int gnca_step_f32(const gnca_step_desc* desc, const gnca_weights* w, const float* x,
                  float* x_out, const void* fire, float* attn, void* ws, size_t ws_bytes,
                  void* stream);

/*
 * One step restricted to the samples with active[b] != 0 (active: uint8 [B], device memory); the
 * other samples are copied through unchanged and do not fire.  Replaces the trainers'
 * `state[mask] = model(state[mask], fire_rate)` variable-length rollout masking
 * (src/training/train_graph_augmented_nca.py:305-321) without the gather/scatter copies of the
 * sub-batch and without a host-side mask.any() sync.  `fire` (GNCA_FIRE_RAND_F32 / MASK_U8) is
 * indexed by the full batch; GNCA_ATTENTION is not supported here.
 */
int gnca_step_masked_f32(const gnca_step_desc* desc, const gnca_weights* w, const float* x,
                         float* x_out, const void* fire, const uint8_t* active, void* ws,
                         size_t ws_bytes, void* stream);

/* Measurement hook: run only the step's kernels named in `phases` (GNCA_PHASE_* bits) with the
 * same arguments as gnca_step_f32.  gnca_step_f32 == all phases.  Skipping a phase leaves its
 * outputs stale; bench.py uses this to time K1 alone with HIP events on `stream`. */
#define GNCA_PHASE_K0 (1u << 0)  /* zero-pad offset weights                */
#define GNCA_PHASE_K1 (1u << 1)  /* perceive + gather + MLP -> dx, partials */
#define GNCA_PHASE_K2 (1u << 2)  /* GroupNorm + residual + alive gate       */
#define GNCA_PHASE_ALL (GNCA_PHASE_K0 | GNCA_PHASE_K1 | GNCA_PHASE_K2)
/* Rollout mode of the measurement hook: K2 writes the next step's alive masks into the workspace
 * and K1 reads them (what gnca_rollout_f32 does for every step after the first; needs
 * 0 <= alpha_thr <= graph_alpha_thr, and a K2 call with this bit on the same workspace first).
 * On a zero-padded-shift graph step with GNCA_PHASE_COMPACT as well, that K2 also hands over the
 * new state's per-(channel, row) sums and the next K0 reads them instead of recomputing them: both
 * calls of such a pair must carry the same flags (a pair that mixes COMPACT and non-COMPACT calls
 * would read stale sums). */
#define GNCA_PHASE_ALIVE (1u << 3)
/* Rollout mode's compact update field (what gnca_rollout_f32 does for every step when the planned
 * K1 is the 16-channel split kernel): K1 writes dx only for its live cells, packed per tile in
 * live-cell order with per-tile-row live masks, and K2 reads them back (dead cells have dx = 0).
 * Both the K1 and the K2 call of a step must carry it; ignored for other K1 variants. */
#define GNCA_PHASE_COMPACT (1u << 4)
int gnca_step_phases_f32(const gnca_step_desc* desc, const gnca_weights* w, const float* x,
                         float* x_out, const void* fire, float* attn, void* ws, size_t ws_bytes,
                         void* stream, uint32_t phases);

/*
 * GraphAugmentation.forward alone: agg_message [B,C,H,W] (before the message policy) and, if
 * GNCA_ATTENTION, the normalised attention map.  Uses desc's graph fields only.
 */
int gnca_message_f32(const gnca_step_desc* desc, const gnca_weights* w, const float* x,
                     float* message, float* attn, void* ws, size_t ws_bytes, void* stream);

/* FixedSobelPerception.forward: y [B,3C,H,W] in the reference's [id.., sobel_x.., sobel_y..] order. */
int gnca_perceive_f32(int32_t B, int32_t C, int32_t H, int32_t W, const float* weight,
                      const float* x, float* y, void* stream);

/*
 * A whole no-grad rollout of `steps` CA steps with GNCA_FIRE_HASH (or GNCA_FIRE_NONE) masks:
 * step t uses offsets[t*2*k .. ] (host array, k = desc->num_offsets pairs per step) and
 * rng_step = desc->rng_step + t.  x is read, x_final receives the last state; scratch holds
 * one more state ([B,C,H,W] fp32).  Equivalent to `steps` gnca_step_f32 calls.  Large batches
 * (gnca_k1_variant's arith bit 4) run as 2 sub-batches of samples, each on its own stream forked
 * from and joined back into `stream` (stream-ordered for the caller, capturable), so that one
 * sub-batch's memory-bound finalize kernel runs on the CUs beside the other's MFMA kernel; the
 * results are bitwise those of one stream.  `ws` then holds one workspace per sub-batch
 * (gnca_workspace_bytes accounts for it).
 */
int gnca_rollout_f32(const gnca_step_desc* desc, const gnca_weights* w, int32_t steps,
                     const int8_t* offsets, const float* x, float* x_final, float* scratch,
                     void* ws, size_t ws_bytes, void* stream);

/*
 * gnca_rollout_f32 in pieces: a long rollout issued as several calls (the host draws the next
 * piece's offsets while the device runs the previous piece) computes exactly the one-call result
 * when the pieces hand the alive masks over through the shared workspace:
 *   GNCA_ROLLOUT_ALIVE_OUT  the last step's K2 also writes the next state's alive masks into `ws`
 *                           (zero-padded shift on the compact field: and its fp64 row sums for K0)
 *   GNCA_ROLLOUT_ALIVE_IN   the first step's K1 reads them from `ws` (written by the previous call
 *                           with ALIVE_OUT on the same workspace; x = that call's x_final)
 * Both need 0 <= alpha_thr <= graph_alpha_thr (else GNCA_ERR_INVALID).  flags = 0 is gnca_rollout_f32.
 * A rollout that runs as concurrent sub-batches (gnca_rollout_f32) forks its helper streams in the
 * first piece and joins them into `stream` in the last one (the piece without ALIVE_OUT): between
 * pieces, x_final is complete on `stream` only for sub-batch 0, so the caller must not read it
 * before the last piece; continuation pieces reuse the first piece's weight images in `ws`.
 */
#define GNCA_ROLLOUT_ALIVE_IN  (1u << 0)
#define GNCA_ROLLOUT_ALIVE_OUT (1u << 1)
/*
 * Rollouts that fold each step's finish into the next step's K1 (gnca_k1_variant's arith bit 8: one
 * K1 launch per step, one K2 at the end) can hand the LAST step over unfinished instead, which
 * saves the K2 and the next piece's plain first K1:
 *   GNCA_ROLLOUT_PENDING_OUT  the last step is left pending: x_final receives the state BEFORE the
 *                             last step and `ws` holds that step's update field
 *   GNCA_ROLLOUT_PENDING_IN   x is such a state and `ws` the pending field of the previous call
 *                             (same desc shape, workspace and stream; desc->rng_step continues the
 *                             previous call's: the field's buffer is chosen by the step's parity)
 * A piece chain PENDING_OUT, PENDING_IN|PENDING_OUT, ..., PENDING_IN computes exactly the one-call
 * rollout.  GNCA_ERR_INVALID when the rollout does not fold, or combined with ALIVE_IN / ALIVE_OUT
 * on the same side.
 */
#define GNCA_ROLLOUT_PENDING_IN  (1u << 2)
#define GNCA_ROLLOUT_PENDING_OUT (1u << 3)
/* Fold even on the compact update field (gnca_k1_variant arith bit 16): large batches otherwise run
 * the two-stream sub-batch pipeline, which measured faster on MI355X ("The fold").
 * Where the request changes the plan (it is not the default for this shape), it is GNCA_ERR_INVALID
 * together with ALIVE_IN / ALIVE_OUT: every piece of an ALIVE chain must run one plan, and a fold
 * chain hands over with PENDING_IN / PENDING_OUT instead. */
#define GNCA_ROLLOUT_FOLD        (1u << 4)
int gnca_rollout_ex_f32(const gnca_step_desc* desc, const gnca_weights* w, int32_t steps,
                        const int8_t* offsets, const float* x, float* x_final, float* scratch,
                        void* ws, size_t ws_bytes, uint32_t flags, void* stream);

/*
 * Measurement twin of gnca_rollout_f32: the same launches, and every K1 / K2 workgroup also writes
 * two wall-clock stamps (the 100 MHz s_memrealtime counter: at its first instruction and after its
 * last barrier) into `stamps` (device memory, uint64, zero-initialised by the caller):
 *   stamps[(((t * nsub + j) * 2 + k) * stamp_cap + wg) * 2 + {0: start, 1: end}],
 *   t = step, j = sub-batch (nsub = 2 when gnca_k1_variant's arith has bit 4, else 1),
 *   k = 0 (K1) / 1 (K2)
 * so a launch's duration is max(end) - min(start) over its workgroups, with no event or marker in
 * the stream between launches.  GNCA_ERR_INVALID if a launch has more than stamp_cap workgroups.
 */
int gnca_rollout_stamped_f32(const gnca_step_desc* desc, const gnca_weights* w, int32_t steps,
                             const int8_t* offsets, const float* x, float* x_final, float* scratch,
                             void* ws, size_t ws_bytes, uint64_t* stamps, int32_t stamp_cap,
                             void* stream);

/*
 * The fire mask a GNCA_FIRE_HASH step would draw: mask[b,0,i,j] = u(rng_seed, rng_step,
 * sample_base+b, i*W+j) <= fire_rate, as uint8 [B,1,H,W] (1 = fires).  For inspection and for
 * replaying a hash-masked rollout elsewhere (e.g. as GNCA_FIRE_MASK_U8).
 */
int gnca_fire_mask_u8(const gnca_step_desc* desc, uint8_t* mask, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Backward (BPTT).  Gradients of one step, written into caller buffers (overwritten, not
 * accumulated), in the reference's parameter layouts.  A NULL pointer skips that gradient's
 * write (e.g. gn_weight/gn_bias without GNCA_USE_GROUPNORM, the graph fields for NeuralCA).
 * -------------------------------------------------------------------------------------------*/
typedef struct gnca_grads {
  float* w1;          /* d update_net.0.weight  [hidden,3C,1,1] */
  float* b1;          /* d update_net.0.bias    [hidden]        */
  float* w2;          /* d update_net.2.weight  [C,hidden,1,1]  */
  float* gn_weight;   /* d norm.weight          [C]             */
  float* gn_bias;     /* d norm.bias            [C]             */
  float* wq;          /* d graph.query_proj.weight [d,C,1,1]    */
  float* bq;          /* d graph.query_proj.bias   [d]          */
  float* wk;          /* d graph.key_proj.weight   [d,C,1,1]    */
  float* bk;          /* d graph.key_proj.bias     [d]          */
  float* wm;          /* d graph.msg_proj.weight   [C,C,1,1]    */
  float* bm;          /* d graph.msg_proj.bias     [C]          */
  float* scaling;     /* d graph.scaling           []           */
} gnca_grads;

/* Bytes of device workspace gnca_step_bwd_f32 needs for `desc` (0 on invalid desc). */
size_t gnca_bwd_workspace_bytes(const gnca_step_desc* desc);

/* Measurement: the backward MLP kernel (BB) the plan for `desc` launches without an active-sample
 * mask, as "gnca_b_mlp<CP,HB,FULL,TH,TW,RY,RX,K,LEAN>" (TH .. K 0 / -1 for the runtime-geometry
 * kernels; NUL-terminated, truncated to n bytes); a masked step never takes the LEAN (24x24) tiles.
 * Host-only.  Returns GNCA_OK or GNCA_ERR_INVALID. */
int gnca_bb_variant(const gnca_step_desc* desc, char* name, int32_t n);

/*
 * Vector-Jacobian product of one step: given the step input x (and the same desc, weights and
 * fire input as the forward call) and gy = dL/d x_out, write gx = dL/dx and the parameter
 * gradients.  The alive / fire masks are constants, the perception weight is frozen (no
 * gradient), as in the reference's autograd graph.  In torus mode the offset weights are exactly
 * uniform, so the query/key/scaling gradients are exactly zero.  gx must not alias x or gy.
 *   active: NULL, or the uint8 [B] sample mask of a gnca_step_masked_f32 forward (inactive
 *           samples: gx = gy, no parameter gradient).
 *   saved: the workspace of the gnca_step_f32 call that produced x_out (same desc, weights, x
 *          and fire), kept unmodified since: its update field and GroupNorm partials are reused.
 *          NULL: the backward recomputes them (one more forward pass).
 */
int gnca_step_bwd_f32(const gnca_step_desc* desc, const gnca_weights* w, const float* x,
                      const void* fire, const uint8_t* active, const float* gy, float* gx,
                      const gnca_grads* grads, const void* saved, void* ws, size_t ws_bytes,
                      void* stream);

/* ---------------------------------------------------------------------------------------------
 * Step-adjacent batch op: damage (src/utils/damage.py:15-138).  ONE damage kind for the whole
 * batch, in place on the [B,C,H,W] state, with the random draws supplied by the caller (device
 * memory), so a whole batch is one launch with no host round trip per sample.
 * -------------------------------------------------------------------------------------------*/
#define GNCA_DMG_SQUARE       0  /* cutout_square_:  zero all channels of [y,y+size) x [x,x+size)      */
#define GNCA_DMG_CIRCLE       1  /* cutout_circle_:  zero all channels where (i-cy)^2+(j-cx)^2 <= r^2  */
#define GNCA_DMG_STRIPE_H     2  /* stripe_wipe_ "h": zero rows [y0, y0+width) (pos[b] = (y0, 0))       */
#define GNCA_DMG_STRIPE_V     3  /* stripe_wipe_ "v": zero cols [x0, x0+width) (pos[b] = (0, x0))       */
#define GNCA_DMG_ALPHA_DROP   4  /* alpha_dropout_(hard): zero all channels where u<p and alpha>thr     */
#define GNCA_DMG_ALPHA_DROP_SOFT 5 /* alpha_dropout_(hard=False): alpha only                            */
#define GNCA_DMG_SALT_PEPPER  6  /* salt_pepper_alpha_: alpha *= (u >= p)                               */
#define GNCA_DMG_GAUSSIAN     7  /* gaussian_hole_: all channels *= clamp(1-exp(-r^2/(2(R*soft)^2)),0,1) */
#define GNCA_DMG_HIDDEN_NOISE 8  /* hidden_scramble_: hidden = clamp(hidden + sigma*n, 0, 1)          */

typedef struct gnca_damage_desc {
  int32_t B, C, H, W;
  int32_t kind;        /* GNCA_DMG_*                                                          */
  int32_t size;        /* square side, circle / gaussian radius, stripe width                  */
  float p;             /* alpha_drop / salt_pepper probability                                 */
  float alpha_thr;     /* alpha_drop: alive threshold                                          */
  float softness;      /* gaussian                                                             */
  float sigma;         /* hidden noise scale                                                   */
} gnca_damage_desc;

/*
 * pos:   int32 [B,2] per-sample (y, x) / centre (cy, cx) for the geometric kinds, else NULL
 * noise: fp32 uniforms [B,1,H,W] (alpha kinds) or normals [B,C-4,H,W] (hidden noise), else NULL
 */
int gnca_damage_f32(const gnca_damage_desc* desc, float* state, const int32_t* pos,
                    const float* noise, void* stream);

/*
 * The graph trainer's loss (src/training/train_graph_augmented_nca.py:52-61), fused:
 *   per_sample[b] = mean_{c<4,i,j} (rgba(pred)[b,c,i,j] - target[b,c,i,j])^2,
 *   rgba(pred) = (pred_rgb * pred_alpha, pred_alpha),
 * and its backward grad_pred[b,c,i,j] = g[b] * d per_sample[b] / d pred[b,c,i,j] (channels 0..3).
 * pred / grad_pred are [B,4,H,W] with sample stride `pred_bstride` floats and channel stride H*W
 * (a channel slice of a contiguous [B,C,H,W] state: pred_bstride = C*H*W); target has sample
 * stride `target_bstride` (0 = one target broadcast over the batch).  fp64 per-sample sums.
 */
int gnca_loss_premult_f32(int32_t B, int32_t H, int32_t W, const float* pred, int64_t pred_bstride,
                          const float* target, int64_t target_bstride, float* per_sample, void* stream);
int gnca_loss_premult_bwd_f32(int32_t B, int32_t H, int32_t W, const float* pred, int64_t pred_bstride,
                              const float* target, int64_t target_bstride, const float* g,
                              float* grad_pred, int64_t grad_bstride, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GNCA_H */
