/* abcd_hip.h -- C ABI of the MI355X (gfx950) ABCD-VAE training path.
 *
 * libabcd_hip.so implements the hot path of the reference trainer
 * (ABCD-VAE/learning.py:147-163: encoder -> sampler -> KL -> decoder -> loss ->
 * backward -> clip_grad_norm_ -> SGD) as hand-written HIP kernels for CDNA4.
 * The reference has no native plugin boundary: its hot path sits behind
 * PyTorch nn.Module methods.  Each entry point below replaces one of those
 * methods (cited per function); the reference-side ctypes binding a
 * maintainer would add is shown in INTEGRATION.md.
 *
 * Conventions
 *   - every pointer is DEVICE memory unless marked HOST;
 *   - all floating point is IEEE fp32 (the reference trains in fp32);
 *   - the packed layout is PyTorch's PackedSequence: rows are time-major,
 *     step t owns rows [off_t, off_t + batch_sizes[t]), batch_sizes is
 *     non-increasing and lives on the HOST (as in PackedSequence);
 *   - `stream` is a hipStream_t (void* here to keep this header HIP-free);
 *     every call is asynchronous and stream-ordered, no host synchronisation;
 *   - the caller owns all memory; `ws` is a caller-allocated workspace of at
 *     least *_workspace_bytes(); the SAME workspace must be passed to the
 *     backward of a module as to its forward (it holds the activation stash);
 *   - return value: 0 on success, a hipError_t code, or ABCD_EINVAL for
 *     unsupported shapes/arguments.  Nothing throws across this ABI.
 *
 * Shape support: the kernels take hidden sizes, MLP width, codebook dim,
 * #categories, speaker embedding dim and the plain feature size in multiples
 * of 16; the frequency-bin count F is arbitrary (padded internally); encoder
 * layers <= 4.  Any other size (the reference accepts every -K, -f and
 * --*_hidden_size, learning.py:371-376) runs as the ZERO-PADDED model: each
 * size rounded up to 16, the real weights embedded at their unit / gate /
 * block positions and every padding weight 0.  Padding units then stay exactly
 * 0 through every recurrence, tanh and product, so values and gradients at the
 * real positions are the real model's; only the categorical softmax needs to
 * know the real sizes (abcd_sampler_cfg.valid_categories / valid_feature_dim).
 * The Python host (modules/padding.py) embeds the parameters and extracts the
 * gradients; INTEGRATION.md shows the index maps.
 */
#ifndef ABCD_HIP_H
#define ABCD_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ABCD_EINVAL 1000
#define ABCD_MAX_LAYERS 4

enum abcd_rnn_type { ABCD_LSTM = 0, ABCD_GRU = 1 };

typedef struct abcd_rnn_w { const float *w_ih, *w_hh, *b_ih, *b_hh; } abcd_rnn_w;
typedef struct abcd_rnn_g { float *w_ih, *w_hh, *b_ih, *b_hh; } abcd_rnn_g;
typedef struct abcd_mlp_w { const float *w1, *b1, *w2, *b2; } abcd_mlp_w; /* Linear->Tanh->Linear */
typedef struct abcd_mlp_g { float *w1, *b1, *w2, *b2; } abcd_mlp_g;

/* A packed batch (torch.nn.utils.rnn.PackedSequence): data is L x F. */
typedef struct abcd_packed {
  const float* data;          /* L x F, may be NULL for the decoder without ground truth */
  const int64_t* batch_sizes; /* HOST, T entries */
  int T, L, B, F;
} abcd_packed;

/* ------------------------------------------------------------------------
 * Encoder: RNN_Variational_Encoder (ABCD-VAE/modules/model.py:40-66)
 * ---------------------------------------------------------------------- */
typedef struct abcd_encoder_cfg {
  int input_size, hidden_size, rnn_type, layers, bidirectional;
} abcd_encoder_cfg;
typedef struct abcd_encoder_params { abcd_rnn_w w[ABCD_MAX_LAYERS][2]; } abcd_encoder_params;
typedef struct abcd_encoder_grads { abcd_rnn_g g[ABCD_MAX_LAYERS][2]; } abcd_encoder_grads;

/* hidden_size_total of model.py:54-58 */
int abcd_encoder_out_size(const abcd_encoder_cfg* cfg);
size_t abcd_encoder_workspace_bytes(const abcd_encoder_cfg* cfg, int T, int L, int B);
/* replaces RNN_Variational_Encoder.forward (model.py:60-66): last_hidden is
 * B x out_size laid out [h_l0f, c_l0f, h_l0b, c_l0b, h_l1f, ...] */
int abcd_encoder_forward(const abcd_encoder_cfg* cfg, const abcd_encoder_params* p, const abcd_packed* x,
                         float* last_hidden, void* ws, size_t ws_bytes, void* stream);
/* autograd backward of the above: writes (overwrites) every weight gradient */
int abcd_encoder_backward(const abcd_encoder_cfg* cfg, const abcd_encoder_params* p, const abcd_packed* x,
                          const float* d_last_hidden, const abcd_encoder_grads* g, void* ws, size_t ws_bytes,
                          void* stream);

/* The same backward with part of the weight-gradient reductions on
 * `wgrad_stream`: for a bidirectional encoder, the first layer's
 * backward-direction weight gradients are reduced on wgrad_stream (forked
 * after the BPTT) beside the forward direction's on `stream`, which then
 * waits for wgrad_stream, so on return every gradient is complete in
 * `stream` order.  wgrad_stream == NULL or == stream: identical to
 * abcd_encoder_backward. */
int abcd_encoder_backward_overlap(const abcd_encoder_cfg* cfg, const abcd_encoder_params* p, const abcd_packed* x,
                                  const float* d_last_hidden, const abcd_encoder_grads* g, void* ws, size_t ws_bytes,
                                  void* stream, void* wgrad_stream);

/* Training-mode inter-layer dropout of nn.LSTM/GRU(dropout = p) (applied by
 * ATen to the packed output of every layer but the last, model.py:53):
 * noise is a HOST array of layers - 1 DEVICE pointers, noise[l] = L x dirs*H
 * values bernoulli(1 - p) / (1 - p) drawn by the caller (in the reference's
 * RNG order for parity, or abcd_fill_dropout); noise == NULL or noise[l] ==
 * NULL: no dropout at that boundary.  The backward takes the same noise. */
int abcd_encoder_forward_dropout(const abcd_encoder_cfg* cfg, const abcd_encoder_params* p, const abcd_packed* x,
                                 const float* const* noise, float* last_hidden, void* ws, size_t ws_bytes,
                                 void* stream);
int abcd_encoder_backward_dropout(const abcd_encoder_cfg* cfg, const abcd_encoder_params* p, const abcd_packed* x,
                                  const float* const* noise, const float* d_last_hidden, const abcd_encoder_grads* g,
                                  void* ws, size_t ws_bytes, void* stream, void* wgrad_stream);
/* The weight gradients of one LSTM layer over its packed frames, every
 * direction at once: the autograd of nn.LSTM's w_ih, b_ih, b_hh, w_hh
 * (model.py:53,60-66) given the gate gradients.  For direction d < nd <= 2:
 *   w_ih[d] = dG[d]^T X,  b_ih[d] = b_hh[d] = colsum(dG[d]),  w_hh[d] = dG[d]^T Hprev[d]
 * dG[d]: K x 4H (row stride 4H, gate blocks i, f, g, o), X: K x F (row
 * stride ldx), Hprev[d]: K x H (stride H; the hidden state each frame's step
 * consumed, zero where it had no predecessor).  b_hh[d] may be NULL.  The
 * encoder backward runs this after its BPTT (layer 0); at F <= 143 with
 * roundup16(F) = 144 and H = 256 it is one gemm_wg3b launch + one slab reduction. */
size_t abcd_lstm_wgrad_workspace_bytes(int nd, int F, int H, int K);
int abcd_lstm_wgrad(int nd, int F, int H, int K, const float* const* dG, const float* X, long ldx,
                    const float* const* Hprev, float* const* w_ih, float* const* b_ih, float* const* b_hh,
                    float* const* w_hh, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * ABCDSampler (model.py:538-639) and the plain Gaussian Sampler
 * (plain/modules/model.py:538-567, model.py:17-28)
 * ---------------------------------------------------------------------- */
typedef struct abcd_sampler_cfg {
  int input_size, mlp_hidden, num_categories, feature_dim;
  int plain; /* 1: plain Gaussian feature sampler (feature_dim = output_size) */
  /* A zero-padded model (every size rounded up to 16, padding weights 0; see
   * "Shape support" above): the model's own category count (the first
   * valid_categories of the num_categories logit columns are categories, the
   * rest are masked out of every softmax, KL and perplexity) and feature dim
   * (the logits scale 1 / sqrt(valid_feature_dim), model.py:589; plain: the
   * feature columns >= valid_feature_dim draw zero noise, so their samples are
   * the padding mean 0).  0: the padded size itself. */
  int valid_categories, valid_feature_dim;
} abcd_sampler_cfg;
typedef struct abcd_sampler_params {
  abcd_mlp_w mlp[2];                 /* ABCD: mlp[0] = to_code_like; plain: mlps.0 (mean), mlps.1 (log-var) */
  const float* codebook;             /* D x K  (ABCD only) */
  const float* posterior_shape_logits; /* K (ABCD only) */
  float prior_concentration;
} abcd_sampler_params;
typedef struct abcd_sampler_grads {
  abcd_mlp_g mlp[2];
  float* codebook;
  float* posterior_shape_logits;
} abcd_sampler_grads;

/* sampling modes */
enum abcd_sample_mode { ABCD_SAMPLE_SOFTMAX = 0, ABCD_SAMPLE_GUMBEL = 1 };

size_t abcd_sampler_workspace_bytes(const abcd_sampler_cfg* cfg, int B);
/* replaces ABCDSampler.forward (model.py:581-590): logits B x K.
 * plain: Sampler.forward -> params_out = [mean | log_var] (B x 2f). */
int abcd_sampler_forward(const abcd_sampler_cfg* cfg, const abcd_sampler_params* p, const float* h, int B,
                         float* logits, void* ws, size_t ws_bytes, void* stream);
/* replaces ABCDSampler.sample (model.py:592-606) / plain Sampler.sample:
 * feats B x D.  noise: ABCD gumbel mode: B x K gumbel g = -log(Exp(1));
 * plain: B x f standard normal.  noise == NULL -> in-kernel Philox(seed, offset). */
int abcd_sampler_sample(const abcd_sampler_cfg* cfg, const abcd_sampler_params* p, const float* logits, int B,
                        int mode, float temperature, const float* noise, uint64_t seed, uint64_t offset,
                        float* feats, void* ws, size_t ws_bytes, void* stream);
/* replaces ABCDSampler.kl_divergence (model.py:608-639) / plain kl: writes a device scalar */
int abcd_sampler_kl(const abcd_sampler_cfg* cfg, const abcd_sampler_params* p, const float* logits, int B,
                    double entire_data_size, float* kl_out, void* ws, size_t ws_bytes, void* stream);
/* forward + sample + kl of one training step (learning.py:149-153 calls
 * feature_sampler(h), .sample(logits), .kl_divergence(logits, N) in turn):
 * logits B x K, feats B x D and the KL scalar (kl_out may be NULL), the same
 * values and backward stash as the three calls above.  ABCD: two launches --
 * the split-K h W1^T GEMM and one row-tiled sampler-head kernel (MLP tail,
 * logits, Gumbel-softmax, y C^T and the KL row terms per 16-row tile, the KL
 * scalar reduced by the last tile).  plain: the three calls in turn.
 * ppl_out (ABCD, may be NULL): ppl_out[0..1] = the cluster and batch
 * perplexities of abcd_perplexities on these logits (reduced by the same
 * last tile); ppl_out[2] is left to abcd_shape_perplexity (it reads
 * posterior_shape_logits after the SGD step, learning.py:171-178). */
/* The Dirichlet prior's per-category terms of ABCDSampler.kl_divergence
 * (model.py:608-639: alpha = softmax(posterior_shape_logits) * N + a0, its
 * digamma / trigamma / lgamma terms) into the workspace stash -- they depend
 * on the parameters only, not on the batch, so a training step can run this
 * one-workgroup kernel on a side stream early and pass
 * mode | ABCD_SAMPLE_PRIOR_READY to abcd_sampler_forward_fused (same ws and
 * B, same entire_data_size, the side stream joined first).  plain: no-op. */
#define ABCD_SAMPLE_PRIOR_READY 0x100
int abcd_sampler_prior(const abcd_sampler_cfg* cfg, const abcd_sampler_params* p, int B, double entire_data_size,
                       void* ws, size_t ws_bytes, void* stream);
int abcd_sampler_forward_fused(const abcd_sampler_cfg* cfg, const abcd_sampler_params* p, const float* h, int B,
                               int mode, float temperature, const float* noise, uint64_t seed, uint64_t offset,
                               double entire_data_size, float* logits, float* feats, float* kl_out, float* ppl_out,
                               void* ws, size_t ws_bytes, void* stream);
/* backward of forward+sample+kl.  d_feats: B x D (may be NULL); d_kl: device
 * scalar upstream grad of kl (may be NULL); d_h: B x E (may be NULL). */
int abcd_sampler_backward(const abcd_sampler_cfg* cfg, const abcd_sampler_params* p, const float* h, int B,
                          int mode, float temperature, double entire_data_size, const float* d_feats,
                          const float* d_kl, float* d_h, const abcd_sampler_grads* g, void* ws, size_t ws_bytes,
                          void* stream);
/* the same, with the parameter gradients (codebook, posterior_shape_logits,
 * MLP weights and biases) queued on wgrad_stream (NULL or == stream: one
 * stream) after an event on `stream`; only the d_h chain stays on `stream`.
 * ABCD with d_feats and d_kl: one row-tiled sampler-head backward kernel
 * (d_logits, dU, dZ1, the bias / prior column sums and d posterior_shape_logits
 * in its last tile) + the d_h GEMM on `stream`; codebook / W2 / W1 GEMMs on
 * wgrad_stream.
 * The caller joins wgrad_stream before reading the gradients.
 * wgrad_stream == ABCD_DEFER_PARAMS (fused ABCD path only): the codebook / W2
 * / W1 gradients are not launched; the caller runs
 * abcd_sampler_backward_params with the same workspace (and h) later -- the
 * training step queues them after the encoder BPTT, off its critical path. */
#define ABCD_DEFER_PARAMS ((void*)(intptr_t)-1)
int abcd_sampler_backward_split(const abcd_sampler_cfg* cfg, const abcd_sampler_params* p, const float* h, int B,
                                int mode, float temperature, double entire_data_size, const float* d_feats,
                                const float* d_kl, float* d_h, const abcd_sampler_grads* g, void* ws,
                                size_t ws_bytes, void* stream, void* wgrad_stream);
/* the deferred codebook / W2 / W1 gradients of a preceding
 * abcd_sampler_backward_split(..., ABCD_DEFER_PARAMS) on `stream`: one
 * batched launch (dC = [d_feats; U]^T [Y; dL / sqrt(D)], dW2 = dU^T Z1,
 * dW1 = dZ1^T h); returns 0 without work when that call took another path
 * (the split call records per workspace whether it deferred; a params call
 * without a matching deferral does nothing).
 * wgrad_stream (NULL or == stream: on `stream`): the launch goes there behind
 * an event on `stream`, in a tiling that co-resides with the encoder's
 * persistent BPTT (the training step queues it on its side stream behind the
 * decoder's weight gradients); the caller joins before reading them. */
int abcd_sampler_backward_params(const abcd_sampler_cfg* cfg, const abcd_sampler_params* p, const float* h, int B,
                                 const abcd_sampler_grads* g, void* ws, size_t ws_bytes, void* stream,
                                 void* wgrad_stream);
/* The same backward split the way autograd sees the three reference methods:
 * sample_backward:  d_feats -> d_logits (written), d_codebook (written, may be NULL)
 *                   (plain: d_feats -> d[mean | log_var])
 * kl_backward:      d_kl -> d_logits (written, or added when accumulate), d_psl (may be NULL)
 * forward_backward: d_logits -> MLP grads, codebook grad of the logits product
 *                   (added to g->codebook when accumulate_codebook), d_h (may be NULL) */
int abcd_sampler_sample_backward(const abcd_sampler_cfg* cfg, const abcd_sampler_params* p, int B, int mode,
                                 float temperature, const float* d_feats, float* d_logits, float* d_codebook,
                                 void* ws, size_t ws_bytes, void* stream);
int abcd_sampler_kl_backward(const abcd_sampler_cfg* cfg, const abcd_sampler_params* p, int B,
                             double entire_data_size, const float* d_kl, int accumulate, float* d_logits,
                             float* d_psl, void* ws, size_t ws_bytes, void* stream);
int abcd_sampler_forward_backward(const abcd_sampler_cfg* cfg, const abcd_sampler_params* p, const float* h, int B,
                                  const float* d_logits, float* d_h, const abcd_sampler_grads* g,
                                  int accumulate_codebook, void* ws, size_t ws_bytes, void* stream);
/* learning.py:171-178 diagnostics: out[0..2] = posterior clustering /
 * batch-mean / Dirichlet-shape perplexities (device floats) */
int abcd_perplexities(const float* logits, int B, int K, const float* posterior_shape_logits, float* out,
                      void* stream);
/* out[0] = exp(entropy of softmax(posterior_shape_logits)) (abcd_perplexities' out[2]) */
int abcd_shape_perplexity(const float* posterior_shape_logits, int K, float* out, void* stream);

/* ------------------------------------------------------------------------
 * Decoder: RNN_Variational_Decoder (model.py:84-196, unidirectional)
 * ---------------------------------------------------------------------- */
typedef struct abcd_decoder_cfg {
  int output_size, hidden_size, mlp_hidden, feature_size, rnn_type;
  int feedback;      /* 1: feed the reparameterised sample back (self_feedback, or eval mode) */
  int num_speakers;  /* 0: no speaker embedding */
  int speaker_dim;
} abcd_decoder_cfg;
typedef struct abcd_decoder_params {
  const float* embed_speaker;  /* num_speakers x speaker_dim or NULL */
  const float *f2h_w, *f2h_b;  /* feature2hidden */
  abcd_mlp_w offset, mu, lv;   /* offset_predictor, emission mlps.0, mlps.1 */
  abcd_rnn_w cell;             /* rnn_cell.cell */
} abcd_decoder_params;
typedef struct abcd_decoder_grads {
  float* embed_speaker;
  float *f2h_w, *f2h_b;
  abcd_mlp_g offset, mu, lv;
  abcd_rnn_g cell;
} abcd_decoder_grads;

size_t abcd_decoder_workspace_bytes(const abcd_decoder_cfg* cfg, int T, int L, int B);
/* replaces RNN_Variational_Decoder.forward (model.py:147-196).
 * features: B x feature_size; speakers: device int64 B (or NULL);
 * gt = ground_truth_out (L x F, or NULL); gt_offset (L, or NULL);
 * eps: L x F standard normals in packed order (or NULL -> Philox(seed,offset));
 * outputs (each may be NULL): flatten_out, mu, log_var (L x F), offset_logits (L);
 * losses[0] = emission NLL, losses[1] = offset BCE (device floats). */
int abcd_decoder_forward(const abcd_decoder_cfg* cfg, const abcd_decoder_params* p, const abcd_packed* x,
                         const float* features, const int64_t* speakers, const float* gt_offset,
                         const float* eps, uint64_t seed, uint64_t offset, float* flatten_out, float* mu,
                         float* log_var, float* offset_logits, float* losses, void* ws, size_t ws_bytes,
                         void* stream);
/* backward w.r.t. losses[0] (scaled by *d_em) and losses[1] (scaled by *d_off);
 * d_em/d_off are device scalars; d_features: B x feature_size (may be NULL).
 * ws must hold the abcd_decoder_forward of the same inputs and parameters
 * (its stashes and its packed weight layouts, transposed ones included). */
int abcd_decoder_backward(const abcd_decoder_cfg* cfg, const abcd_decoder_params* p, const abcd_packed* x,
                          const float* features, const int64_t* speakers, const float* gt_offset,
                          const float* d_em, const float* d_off, float* d_features,
                          const abcd_decoder_grads* g, void* ws, size_t ws_bytes, void* stream);
/* The same backward with the weight-gradient reductions (K = all packed
 * frames) moved to `wgrad_stream`: d_features is complete in `stream` order
 * on return (so the sampler/encoder backward can follow on `stream` at once),
 * the weight gradients only in `wgrad_stream` order -- the caller joins the
 * two streams before reading them (e.g. before clip_grad_norm_).  The
 * weight-gradient kernels use a tiling that co-resides with the encoder's
 * persistent BPTT kernel.  wgrad_stream == NULL or == stream: identical to
 * abcd_decoder_backward. */
int abcd_decoder_backward_overlap(const abcd_decoder_cfg* cfg, const abcd_decoder_params* p, const abcd_packed* x,
                                  const float* features, const int64_t* speakers, const float* gt_offset,
                                  const float* d_em, const float* d_off, float* d_features,
                                  const abcd_decoder_grads* g, void* ws, size_t ws_bytes, void* stream,
                                  void* wgrad_stream);
/* Training-mode decoder input dropout (RNN_Cell's nn.Dropout, model.py:289,297):
 * xmask is L x F (DEVICE, packed order) holding bernoulli(1-p)/(1-p) -- the
 * noise the dropout applies to step t's cell input at rows off[t] .. off[t]+bs_t
 * (row block 0 multiplies the zero initial input and only keeps the RNG
 * order).  The sample fed back is mask * x; flatten_out keeps x.  The
 * backward needs the same xmask.  xmask == NULL: no dropout (eval mode,
 * p = 0); cfg->feedback must be 1 when xmask is given. */
int abcd_decoder_forward_dropout(const abcd_decoder_cfg* cfg, const abcd_decoder_params* p, const abcd_packed* x,
                                 const float* features, const int64_t* speakers, const float* gt_offset,
                                 const float* eps, const float* xmask, uint64_t seed, uint64_t offset,
                                 float* flatten_out, float* mu, float* log_var, float* offset_logits, float* losses,
                                 void* ws, size_t ws_bytes, void* stream);
/* the same, with the loss reductions (emission NLL, offset BCE sum -> losses)
 * queued on loss_stream (NULL or == stream: one stream) after events on
 * `stream`; the caller joins loss_stream before reading `losses`. */
int abcd_decoder_forward_split(const abcd_decoder_cfg* cfg, const abcd_decoder_params* p, const abcd_packed* x,
                               const float* features, const int64_t* speakers, const float* gt_offset,
                               const float* eps, const float* xmask, uint64_t seed, uint64_t offset,
                               float* flatten_out, float* mu, float* log_var, float* offset_logits, float* losses,
                               void* ws, size_t ws_bytes, void* stream, void* loss_stream);
/* wgrad_stream == ABCD_DEFER_PARAMS: only the data-gradient part (offset head,
 * BPTT, initial-state / feature gradients: d_features complete in `stream`
 * order); the weight gradients are queued by abcd_decoder_backward_params
 * with the SAME arguments later on this host thread (the training step calls
 * it after queuing the sampler and encoder backward). */
int abcd_decoder_backward_dropout(const abcd_decoder_cfg* cfg, const abcd_decoder_params* p, const abcd_packed* x,
                                  const float* features, const int64_t* speakers, const float* gt_offset,
                                  const float* xmask, const float* d_em, const float* d_off, float* d_features,
                                  const abcd_decoder_grads* g, void* ws, size_t ws_bytes, void* stream,
                                  void* wgrad_stream);
/* the deferred weight gradients of the preceding
 * abcd_decoder_backward_dropout(..., ABCD_DEFER_PARAMS) (same arguments): on
 * wgrad_stream (NULL or == stream: on `stream`) behind an event recorded at the
 * end of that call's data path, in the tiling that co-resides with the
 * encoder's persistent BPTT; with the side-stream gate on, behind a wait for
 * the encoder BPTT launched in between to be resident.  The caller joins
 * wgrad_stream before reading the gradients. */
int abcd_decoder_backward_params(const abcd_decoder_cfg* cfg, const abcd_decoder_params* p, const abcd_packed* x,
                                 const float* features, const int64_t* speakers, const float* gt_offset,
                                 const float* xmask, const float* d_em, const float* d_off, float* d_features,
                                 const abcd_decoder_grads* g, void* ws, size_t ws_bytes, void* stream,
                                 void* wgrad_stream);

/* ------------------------------------------------------------------------
 * Featurisation + packing on the device: replaces the per-item host path
 * Dataset.__getitem__ -> STFT.__call__ -> log_and_normalize -> pack_sequence
 * (data_utils.py:88-103, 124-139, 165-182; learning.py:466-470) for a whole
 * batch.  wave: concatenated fp32 samples (DEVICE); seg_off / seg_len: HOST,
 * one entry per segment in packed (length-descending) order; window: n_fft
 * floats (DEVICE, e.g. torch.hann_window); batch_sizes: HOST, T entries,
 * consistent with the per-segment frame counts.  out: L x (n_fft/2 + 1)
 * packed log-amplitudes log(|STFT| + eps) / norm; is_offset: L (may be NULL),
 * 1 at each segment's last frame.
 * ---------------------------------------------------------------------- */
/* frames torch.stft produces for `length` samples (0 if none) */
int abcd_stft_frames(long long length, int n_fft, int hop, int center);
size_t abcd_featurize_workspace_bytes(int B, int T);
int abcd_featurize_packed(const float* wave, const long long* seg_off, const long long* seg_len, int B, int n_fft,
                          int hop, int center, const float* window, float eps, float norm,
                          const int64_t* batch_sizes, int T, int L, float* out, float* is_offset, void* ws,
                          size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Optimiser: torch.nn.utils.clip_grad_norm_ + torch.optim.SGD
 * (learning.py:161-163, 256) over one flat fp32 parameter/gradient buffer.
 * ---------------------------------------------------------------------- */
size_t abcd_optim_workspace_bytes(long n);
/* The norm's last-block hand-over uses one device-wide ticket word (as do the
 * sampler-head kernels of abcd_sampler_forward_fused / abcd_sampler_backward*):
 * launches of these entry points on one device must not run concurrently on
 * different streams (the training step queues them on one stream). */
/* total 2-norm of g (device scalar) */
int abcd_grad_norm(const float* g, long n, float* out_norm, void* ws, size_t ws_bytes, void* stream);
/* g *= min(1, max_norm / (||g|| + 1e-6)); buf = momentum*buf + g (buf = g if
 * momentum_init); p -= lr * (momentum ? buf : g).  out_norm (device, may be
 * NULL) receives the pre-clip norm. */
int abcd_clip_sgd(float* p, float* g, float* momentum_buf, long n, float max_norm, float lr, float momentum,
                  int momentum_init, float* out_norm, void* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Utilities
 * ---------------------------------------------------------------------- */
/* loss = (losses[0] + losses[1] + kl[0]) / B  (learning.py:155-157) */
int abcd_total_loss(const float* losses, const float* kl, int B, float* loss, void* stream);
/* C = A(MxK) @ B(NxK)^T (+bias[n]); row-major, plain GEMM used by tests */
int abcd_gemm_nt(int M, int N, int K, const float* A, long lda, const float* B, long ldb, float* C, long ldc,
                 const float* bias, void* ws, size_t ws_bytes, void* stream);
/* C = A^T @ B, A K x M (lda >= M), B K x N (ldb >= N), row-major: the
 * weight-gradient GEMM (reduction over packed frames); ws enables split-K
 * (>= 16 * M * N * 4 bytes recommended) */
int abcd_gemm_tn(int M, int N, int K, const float* A, long lda, const float* B, long ldb, float* C, long ldc,
                 void* ws, size_t ws_bytes, void* stream);
/* y = act(x @ W^T + b): nn.Linear (act 0) / Linear->Tanh (act 1); x M x K, W N x K.
 * Used by the standalone MLP modules (model.py:316-334) outside the training step;
 * ws >= (M + N) * roundup(K,16) * 4 bytes when K is not a multiple of 16. */
int abcd_linear(int M, int N, int K, const float* x, long ldx, const float* W, long ldw, const float* b, int act,
                float* y, long ldy, void* ws, size_t ws_bytes, void* stream);
/* backward of abcd_linear (the standalone MLP's training path, model.py:316-334):
 * dy' = dy (act 0) or dy (1 - y^2) (act 1, y = the forward's output);
 * dx = dy' W (M x K, may be NULL), dW = dy'^T x (N x K, row stride K, may be
 * NULL), db = column sums of dy' (N, may be NULL).  Any M, N, K. */
size_t abcd_linear_backward_workspace_bytes(int M, int N, int K);
int abcd_linear_backward(int M, int N, int K, const float* x, long ldx, const float* W, long ldw, const float* y,
                         long ldy, int act, const float* dy, long lddy, float* dx, long lddx, float* dW, float* db,
                         void* ws, size_t ws_bytes, void* stream);
/* n standard normals from Philox-4x32-10(seed, offset + i) */
int abcd_fill_normal(float* out, long n, uint64_t seed, uint64_t offset, void* stream);
/* dropout noise bernoulli(1 - p) / (1 - p) from the same Philox stream */
int abcd_fill_dropout(float* out, long n, float p, uint64_t seed, uint64_t offset, void* stream);
/* live device timing of the recurrent kernel family (encoder and decoder,
 * persistent or per-step): HIP events around every launch while enabled;
 * read: out[0] = summed device ms, out[1] = number of launches */
void abcd_timing_enable(int on);
void abcd_timing_reset(void);
int abcd_timing_read(double* out);
/* the same for one kernel: 0 per-step recurrent kernels, 1 encoder forward,
 * 2 encoder backward, 3 decoder forward, 4 decoder backward (persistent) */
int abcd_timing_read_kernel(int kid, double* out);
/* which kernel the last launch of a role ran (same ids as abcd_timing_read_kernel,
 * 5 / 6 the sampler head forward / backward, 7 the encoder's layer-0 weight
 * gradients; e.g. "dec_bwd_sk<9,16,16,LSTM> grid 256" or "per-step ..."), and how many
 * launches of the role since abcd_dispatch_reset; host-side bookkeeping only */
const char* abcd_dispatch_name(int kid);
long abcd_dispatch_count(int kid);
void abcd_dispatch_reset(void);
/* diagnostics (scripts/, not part of the reference's interface):
 * abcd_debug_persist_prof -- the persistent kernels of the roles in `mask`
 * (1 enc fwd, 2 enc bwd, 4 dec fwd, 8 dec bwd) stamp s_memrealtime at their
 * phase boundaries into dev_buf (blocks x T x 8 u64; null: off); 16 / 32:
 * the sampler-head forward / backward kernels (tiles x 8 u64);
 * abcd_debug_xcc_map -- launches `blocks` one-per-CU workgroups that record
 * their (XCC id, HW_ID) pair into dev_out[2 * block], dev_out[2 * block + 1]
 * (dev_out holds 2 * blocks u32; the placement the persistent kernels' group
 * roles rely on).  Returns 0 / a HIP error. */
void abcd_debug_persist_prof(unsigned long long* dev_buf, int mask);
/* Side-stream gate (per calling host thread, default off): read by a deferred
 * abcd_decoder_backward_dropout(..., ABCD_DEFER_PARAMS).  The first encoder
 * BPTT this thread launches persistently after it becomes the gate's target,
 * and the abcd_decoder_backward_params call that follows queues, in front of
 * its side-stream work, a wait (on the device, bounded) until every workgroup
 * of that launch is resident -- without it the side GEMMs can take a CU's
 * room before a BPTT member is placed there.  No persistent BPTT in between
 * (a per-step encoder backward): no wait.  The wait is queued after the
 * BPTT's launch, so a side stream that shares the BPTT's hardware queue
 * cannot hold the BPTT back. */
void abcd_side_gate_enable(int on);
int abcd_debug_xcc_map(unsigned* dev_out, int blocks, void* stream);
/* 0 if no persistent recurrent kernel has timed out waiting for its group
 * since the last call (a timeout means the grid was not co-resident; the
 * results of that launch are invalid).  Reads and clears the device word;
 * synchronises the device.  Returns -1 on a HIP error. */
int abcd_device_status(void);
/* stream-ordered form for the training step (no host sync): out[0] = the
 * timeout status raised since the previous call (0 ok, 1 a persistent kernel's
 * hand-off wait timed out, 2 a side-stream gate timed out; non-zero means
 * that step's results are invalid), then clears it.  The trainer and bench.py
 * raise on a non-zero value. */
int abcd_step_status(float* out, void* stream);
/* library build identification (gfx target, version) */
const char* abcd_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ABCD_HIP_H */
