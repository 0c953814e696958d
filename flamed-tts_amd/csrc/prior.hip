// Prior transformer stack of PriorGenerator.sample on gfx950: the phoneme encoder,
// the bridge, the shared decoder, the six prompt-prefixed per-quantizer decoders and the code head.
// Reference: flamed/models/synthesizer/prior_generator.py:12-26 (PreEncoding), :141-196 (sample);
// flamed/models/module/transformer/Models.py:10-30 (sinusoid table), :33-100 (Encoder), :103-171
// (Decoder); Layers.py:11-30 (FFTBlock); SubLayers.py:8-57 (MultiHeadAttention, post-norm), :60-95
// (PositionwiseFeedForward); Modules.py:6-25 (ScaledDotProductAttention).
//
// Exact fp32 by default (f32 MFMA GEMMs = fp32 FMA chains; the encoder output feeds the duration flow,
// whose rounded frame counts must match the reference, so the ENCODER always stays fp32).  The decoder
// side (bridge, shared decoder, the six prompt-prefixed decoders, head) may run its GEMMs on bf16
// operands with fp32 accumulation (flamed_prior_set_dtype: weights converted once into a second arena,
// fp32 activations rounded to bf16 in the GEMM A loaders; LayerNorm, softmax, residuals stay fp32).  Rows are channels-last (B*n, D).  Per FFT block
// (7 launches):
//   qkv GEMM   X -> [Q|K|V] (M x 3D), w_qs/w_ks/w_vs packed as one (3D x D) weight
//   attention  one workgroup per (64 queries, head, utterance): K/V staged through LDS in 64-key chunks,
//              each wave runs an online softmax over a quarter of every chunk, the four partial
//              (max, sum, acc) states are merged through LDS; key-padding mask -> -inf (Modules.py:19)
//   fc GEMM    + bias + residual -> R
//   LN + mask  R -> X = LayerNorm(R)*g + b, padded rows 0 (Layers.py:26)
//   conv1 GEMM Conv1d(D->F, k0, pad k0/2) as a tap-gather GEMM + bias + ReLU -> Hf
//   conv2 GEMM Conv1d(F->D, k1) + bias + residual X -> R
//   LN + mask  R -> X (the last block of a decoder also writes its target rows into prior_embs)
#include "flamed_hip.h"
#include "gemm.hpp"
#include "xfmr.hpp"

#include <cmath>
#include <type_traits>
#include <mutex>
#include <vector>

namespace fl {

// ------------------------------------------------------------------ kernels

// conv weight (N, Cin, KT) -> (N, KT, Cin) (K index = tap*Cin + c)
__global__ void prior_taps_kernel(const float* __restrict__ src, float* __restrict__ dst, int N, int Cin, int KT) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t total = (size_t)N * Cin * KT;
  if (i >= total) return;
  int k = i % KT;
  size_t t = i / KT;
  int c = t % Cin;
  int n = t / Cin;
  dst[((size_t)n * KT + k) * Cin + c] = src[i];
}

__global__ void prior_f32_to_bf16_kernel(const float* __restrict__ src, bf16* __restrict__ dst, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (bf16)src[i];
}

// Encoder input: src_word_emb(ids) + position_enc[l] (Models.py:88-92).
__global__ void embed_pos_kernel(const int64_t* __restrict__ ids, const float* __restrict__ emb,
                                 const float* __restrict__ pos, int M, int n, int D, float* __restrict__ X) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;  // float4 index
  int D4 = D >> 2;
  if (i >= M * D4) return;
  int m = i / D4, c = (i - m * D4) * 4;
  float4 e = ld4(emb + (size_t)ids[m] * D + c);
  float4 p = ld4(pos + (size_t)(m % n) * D + c);
  *reinterpret_cast<float4*>(X + (size_t)m * D + c) = make_float4(e.x + p.x, e.y + p.y, e.z + p.z, e.w + p.w);
}

// Decoder q's input (prior_generator.py:178-180 + PreEncoding :21-26 + Decoder :156-158):
//   x[b][j] = ((src + seg) + quantizer_emb[q]) + position_enc[j],  j < P: src = code_embedding(prompt),
//   seg = prompt_emb; j >= P: src = previous decoder's target row j - P, seg = target_emb.
// Also writes the decoder key mask get_mask_from_lengths(P + tgt_len, P + T) as (j >= P) & tgt_mask.
__global__ void dec_input_kernel(const float* __restrict__ prev, int prev_bstride, const int64_t* __restrict__ prompts,
                                 const float* __restrict__ cemb, const float* __restrict__ pemb,
                                 const float* __restrict__ temb, const float* __restrict__ qemb,
                                 const float* __restrict__ pos, const uint8_t* __restrict__ tmask, int B, int P,
                                 int T, int D, int nq, int q, float* __restrict__ X, uint8_t* __restrict__ dmask) {
  const int n = P + T, D4 = D >> 2;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * n * D4) return;
  int row = i / D4, c = (i - row * D4) * 4;
  int b = row / n, j = row - b * n;
  const float* src;
  const float* seg;
  if (j < P) {
    src = cemb + (size_t)prompts[((size_t)b * nq + q) * P + j] * D;
    seg = pemb;
  } else {
    src = prev + ((size_t)b * prev_bstride + (j - P)) * D;
    seg = temb;
  }
  float4 s = ld4(src + c), g = ld4(seg + c), qe = ld4(qemb + c), p = ld4(pos + (size_t)j * D + c);
  float4 o = make_float4(((s.x + g.x) + qe.x) + p.x, ((s.y + g.y) + qe.y) + p.y, ((s.z + g.z) + qe.z) + p.z,
                         ((s.w + g.w) + qe.w) + p.w);
  *reinterpret_cast<float4*>(X + (size_t)row * D + c) = o;
  if (c == 0) dmask[row] = j < P ? 0 : tmask[(size_t)b * T + (j - P)];
}

// bridge(x) + position_enc[l] of the shared decoder (prior_generator.py:167 + Models.py:156-158)
struct EpiBiasPos {
  const float* __restrict__ bias;
  const float* __restrict__ pos;
  int n;
  float* __restrict__ out;
  int ldo;
  static constexpr bool kRowStats = false;
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ float value(int m, int c, float acc, const float*, int) const {
    return (acc + bias[c]) + pos[(size_t)(m % n) * ldo + c];
  }
  __device__ void store(int m, int c, float v) const { out[(size_t)m * ldo + c] = v; }
  __device__ void store4(int m, int c, const float* v) const { store_val4<float>(out + (size_t)m * ldo + c, v); }
  __device__ void store_stats(int, int, float, float) const {}
};

// head(embs) * ~tgt_mask, permuted to (B, V1, nq, T) (prior_generator.py:186-188).  Row m = (b, q, t);
// the weight is zero-padded to a multiple of 64 rows, columns >= V1 are not stored.
struct EpiHead {
  const float* __restrict__ bias;
  const uint8_t* __restrict__ tmask;
  float* __restrict__ out;
  int V1, nq, T;
  static constexpr bool kRowStats = false;
  static constexpr int stat_rows(int) { return 0; }
  __device__ void prologue(int, int, int, float*) const {}
  __device__ float value(int, int n, float acc, const float*, int) const { return acc + bias[n]; }
  __device__ void store(int m, int n, float v) const {
    if (n >= V1) return;
    const int qt = nq * T;
    const int b = m / qt, r = m - b * qt;
    const int q = r / T, t = r - q * T;
    out[(((size_t)b * V1 + n) * nq + q) * T + t] = v * (tmask[(size_t)b * T + t] ? 0.f : 1.f);
  }
  __device__ void store4(int m, int n, const float* v) const {
    for (int j = 0; j < 4; ++j) store(m, n + j, v[j]);
  }
  __device__ void store_stats(int, int, float, float) const {}
};

// ------------------------------------------------------------------ handle

struct FftLayer {
  const float *wqkv, *bqkv, *wfc, *bfc, *g1, *b1, *w1, *c1b, *w2, *c2b, *g2, *b2;
  const bf16 *wqkv16 = nullptr, *wfc16 = nullptr, *w1_16 = nullptr, *w2_16 = nullptr;  // decoder side, bf16 mode
};
struct FftStack {
  int D = 0, H = 0, F = 0, k0 = 0, k1 = 0, maxseq = 0;
  const float* pos = nullptr;  // (maxseq + 1) x D
  std::vector<FftLayer> layers;
};

struct Prior {
  int n_sym = 0, vocab = 0, nq = 0;
  int device = -1;
  std::mutex mu;
  char* dev = nullptr;
  FftStack enc, shared;
  std::vector<FftStack> dec;
  const float *src_emb = nullptr, *bridge_w = nullptr, *bridge_b = nullptr, *code_emb = nullptr;
  const float *prompt_emb = nullptr, *target_emb = nullptr, *q_emb = nullptr, *head_w = nullptr, *head_b = nullptr;
  int head_n = 0;  // padded head rows (multiple of 64)
  CapGraph genc, gdec;
  int dec_dt = FLAMED_F32;  // decoder-side GEMM operands (flamed_prior_set_dtype)
  char* dev16 = nullptr;    // bf16 copies of the decoder-side GEMM weights (made on first bf16 decode)
  const bf16 *bridge_w16 = nullptr, *head_w16 = nullptr;
  // bf16 decoders: split-K of the GEMMs whose tile grid leaves CUs idle (conv2 and fc: N = 384 at 640
  // rows, 240 tiles of K = 1536 / 384), slices summed by the last arriver in a fixed order
  SplitCtx split;
  char* split_mem = nullptr;
  static constexpr int kSplitTarget = 512, kSplitCounters = 2048;
};

static size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }
constexpr int kLayerW = 16;

static int n_weights(const Prior* p) {
  int n = 2 + kLayerW * (int)p->enc.layers.size();            // src_word_emb, encoder.position_enc, layers
  n += 3;                                                      // bridge.{weight,bias}, code_embedding.weight
  n += 1 + kLayerW * (int)p->shared.layers.size();             // shared_decoder.position_enc, layers
  n += 3;                                                      // pre_encode.{prompt_emb,target_emb,quantizer_emb.weight}
  for (const FftStack& s : p->dec) n += 1 + kLayerW * (int)s.layers.size();
  return n + 2;                                                // head.{weight,bias}
}

struct PriorWs {
  float *X, *QKV, *O, *R, *Hf, *Xs;
  uint8_t* dmask;
};
// One layout serves both calls: rows = max(B*L, B*(P+T)) at the widest stack's dims.
static size_t prior_ws_layout(const Prior* p, int B, int L, int T, int P, void* base, PriorWs* w) {
  const size_t Me = (size_t)B * L, Md = (size_t)B * (P + T);
  auto mx = [](size_t a, size_t b) { return a > b ? a : b; };
  const size_t xD = mx(Me * p->enc.D, Md * p->shared.D);
  const size_t xF = mx(Me * p->enc.F, Md * p->shared.F);
  size_t sizes[7] = {4 * xD, 12 * xD, 4 * xD, 4 * xD, 4 * xF, 4ull * B * T * p->shared.D, Md + 64};
  size_t off = 0;
  char* q[7];
  for (int i = 0; i < 7; ++i) {
    q[i] = base ? (char*)base + off : nullptr;
    off += a256(sizes[i]);
  }
  if (w) *w = PriorWs{(float*)q[0], (float*)q[1], (float*)q[2], (float*)q[3], (float*)q[4], (float*)q[5], (uint8_t*)q[6]};
  return off;
}

// One FFTBlock stack (Models.py:94-98 / :160-169) in place on X (M = B*n rows).  `embs` (decoders): the
// last block's LN also writes the target rows into prior_embs[:, q].
// The GEMM weights of a layer in the stack's operand type.
template <typename DT> struct LW;
template <> struct LW<float> {
  static const float* qkv(const FftLayer& l) { return l.wqkv; }
  static const float* fc(const FftLayer& l) { return l.wfc; }
  static const float* c1(const FftLayer& l) { return l.w1; }
  static const float* c2(const FftLayer& l) { return l.w2; }
};
template <> struct LW<bf16> {
  static const bf16* qkv(const FftLayer& l) { return l.wqkv16; }
  static const bf16* fc(const FftLayer& l) { return l.wfc16; }
  static const bf16* c1(const FftLayer& l) { return l.w1_16; }
  static const bf16* c2(const FftLayer& l) { return l.w2_16; }
};
// fp32: the transformer stacks' config choice (xf_gemm); bf16: the shape-driven bf16 configs, with the
// same 32 x 32 tiles when 32 x 64 would leave CUs idle (N = 384 at 640 rows: 120 -> 240 workgroups).
template <typename DT, class AL, class EP>
static int pr_gemm(const AL& al, const DT* W, int ldw, const EP& ep, int M, int N, int K, hipStream_t st) {
  if constexpr (std::is_same<DT, float>::value) {
    return xf_gemm(al, W, ldw, ep, M, N, K, st);
  } else {
    if (M < 2048 && (size_t)(N / 64) * ((M + 31) / 32) < 256 && N % 32 == 0)
      return launch_gemm_cfg<32, 32, 3, bf16>(al, W, ldw, ep, M, N, K, st);
    return launch_gemm<bf16>(al, W, ldw, ep, M, N, K, st);
  }
}

template <typename DT>
static int fft_forward(const FftStack& s, float* X, const uint8_t* mask, int B, int n, const PriorWs& w, hipStream_t st,
                       float* embs = nullptr, int P = 0, int T = 0, int nq = 0, int q = 0) {
  const int M = B * n, D = s.D, F = s.F;
  int rc;
  for (size_t li = 0; li < s.layers.size(); ++li) {
    const FftLayer& Ly = s.layers[li];
    if ((rc = pr_gemm<DT>(LoadF32<DT>{X, D}, LW<DT>::qkv(Ly), D, EpiBiasAct<float, 0>{Ly.bqkv, w.QKV, 3 * D}, M, 3 * D, D, st)))
      return rc;
    if ((rc = attention(D / s.H, w.QKV, mask, B, n, D, s.H, w.O, st))) return rc;
    if ((rc = pr_gemm<DT>(LoadF32<DT>{w.O, D}, LW<DT>::fc(Ly), D, EpiBiasRes{Ly.bfc, X, w.R, D}, M, D, D, st))) return rc;
    if ((rc = ln_mask(D, w.R, Ly.g1, Ly.b1, mask, X, M, n, nullptr, 0, 0, 0, 0, st))) return rc;
    if ((rc = pr_gemm<DT>(LoadConvRows<DT, false>{X, D, n, s.k0, 1, nullptr, 0, 0, 0.f, nullptr, nullptr}, LW<DT>::c1(Ly),
                          s.k0 * D, EpiBiasAct<float, 3>{Ly.c1b, w.Hf, F}, M, F, s.k0 * D, st)))
      return rc;
    if ((rc = pr_gemm<DT>(LoadConvRows<DT, false>{w.Hf, F, n, s.k1, 1, nullptr, 0, 0, 0.f, nullptr, nullptr}, LW<DT>::c2(Ly),
                          s.k1 * F, EpiBiasRes{Ly.c2b, X, w.R, D}, M, D, s.k1 * F, st)))
      return rc;
    const bool last = li + 1 == s.layers.size();
    if ((rc = ln_mask(D, w.R, Ly.g2, Ly.b2, mask, X, M, n, last ? embs : nullptr, P, T, nq, q, st))) return rc;
  }
  return kOk;
}

static int run_encode(Prior* p, const int64_t* texts, const uint8_t* mask, int B, int L, const float* pos, float* out,
                      const PriorWs& w, hipStream_t st) {
  const int D = p->enc.D, M = B * L;
  hipLaunchKernelGGL(embed_pos_kernel, dim3((M * (D / 4) + 255) / 256), dim3(256), 0, st, texts, p->src_emb,
                     pos ? pos : p->enc.pos, M, L, D, out);
  FL_LAUNCH_CHECK();
  return fft_forward<float>(p->enc, out, mask, B, L, w, st);
}

template <typename DT> static const DT* bridge_of(const Prior* p);
template <> const float* bridge_of<float>(const Prior* p) { return p->bridge_w; }
template <> const bf16* bridge_of<bf16>(const Prior* p) { return p->bridge_w16; }
template <typename DT> static const DT* head_of(const Prior* p);
template <> const float* head_of<float>(const Prior* p) { return p->head_w; }
template <> const bf16* head_of<bf16>(const Prior* p) { return p->head_w16; }

template <typename DT>
static int run_decode(Prior* p, const float* x, const uint8_t* tmask, const int64_t* prompts, int B, int T, int P,
                      const float* pos, float* embs, float* logits, const PriorWs& w, hipStream_t st) {
  const int De = p->enc.D, D = p->shared.D, nq = p->nq;
  int rc;
  // bridge + shared decoder (prior_generator.py:165-168)
  if ((rc = pr_gemm<DT>(LoadF32<DT>{x, De}, bridge_of<DT>(p), De,
                        EpiBiasPos{p->bridge_b, pos ? pos : p->shared.pos, T, w.Xs, D}, B * T, D, De, st)))
    return rc;
  if ((rc = fft_forward<DT>(p->shared, w.Xs, tmask, B, T, w, st))) return rc;
  // six chained prompt-prefixed decoders (:172-182)
  const int n = P + T, G = B * n * (D / 4);
  for (int q = 0; q < nq; ++q) {
    const float* prev = q == 0 ? w.Xs : embs + (size_t)(q - 1) * T * D;
    const int pbs = q == 0 ? T : nq * T;
    hipLaunchKernelGGL(dec_input_kernel, dim3((G + 255) / 256), dim3(256), 0, st, prev, pbs, prompts, p->code_emb,
                       p->prompt_emb, p->target_emb, p->q_emb + (size_t)q * D, pos ? pos : p->dec[q].pos, tmask, B, P, T,
                       D, nq, q, w.X, w.dmask);
    FL_LAUNCH_CHECK();
    if ((rc = fft_forward<DT>(p->dec[q], w.X, w.dmask, B, n, w, st, embs, P, T, nq, q))) return rc;
  }
  // code head over (B, nq, T) rows, masked and permuted (:186-188)
  return pr_gemm<DT>(LoadF32<DT>{embs, D}, head_of<DT>(p), D, EpiHead{p->head_b, tmask, logits, p->vocab + 1, nq, T},
                     B * nq * T, p->head_n, D, st);
}

// bf16 copies of every decoder-side GEMM weight (bridge, shared + per-quantizer decoder layers, padded
// head), converted once from the fp32 arena into a second one.
static int ensure_bf16(Prior* p, hipStream_t st) {
  if (p->dev16) return kOk;
  struct Item { const float* src; size_t n; const bf16** dst; };
  std::vector<Item> items;
  const size_t D = p->shared.D, F = p->shared.F, De = p->enc.D;
  items.push_back({p->bridge_w, D * De, &p->bridge_w16});
  auto stack = [&](FftStack& s) {
    for (FftLayer& L : s.layers) {
      items.push_back({L.wqkv, 3 * D * D, &L.wqkv16});
      items.push_back({L.wfc, D * D, &L.wfc16});
      items.push_back({L.w1, F * s.k0 * D, &L.w1_16});
      items.push_back({L.w2, D * s.k1 * F, &L.w2_16});
    }
  };
  stack(p->shared);
  for (FftStack& s : p->dec) stack(s);
  items.push_back({p->head_w, (size_t)p->head_n * D, &p->head_w16});
  if (!p->split_mem) {  // slab: up to kSplitTarget workgroups of 32 x 64 fp32 tiles; zeroed tile counters
    const size_t slab_floats = (size_t)Prior::kSplitTarget * 32 * 64;
    FL_HIP(hipMalloc(&p->split_mem, 4 * slab_floats + 4 * Prior::kSplitCounters));
    FL_HIP(hipMemsetAsync(p->split_mem + 4 * slab_floats, 0, 4 * Prior::kSplitCounters, st));
    p->split.slab = reinterpret_cast<float*>(p->split_mem);
    p->split.slab_floats = slab_floats;
    p->split.cnt = reinterpret_cast<int*>(p->split_mem + 4 * slab_floats);
    p->split.cnt_n = Prior::kSplitCounters;
    p->split.target = Prior::kSplitTarget;
    p->split.max_split = 4;
  }
  size_t total = 0;
  for (const Item& it : items) total += a256(2 * it.n);
  FL_HIP(hipMalloc(&p->dev16, total));
  size_t off = 0;
  for (const Item& it : items) {
    bf16* dst = reinterpret_cast<bf16*>(p->dev16 + off);
    hipLaunchKernelGGL(prior_f32_to_bf16_kernel, dim3((unsigned)((it.n + 255) / 256)), dim3(256), 0, st, it.src, dst, it.n);
    FL_LAUNCH_CHECK();
    *it.dst = dst;
    off += a256(2 * it.n);
  }
  return kOk;
}

}  // namespace fl

using namespace fl;

extern "C" {

FLAMED_API int flamed_prior_create(const int* d, int nd, flamed_prior_t* out) {
  FL_REQUIRE(out && d && nd >= 17, "flamed_prior_create: need at least 17 dims");
  const int nq = d[16];
  FL_REQUIRE(nq >= 1 && nd == 17 + nq, "flamed_prior_create: expected %d dims for %d quantizers", 17 + nq, nq);
  auto ok_stack = [](int D, int H, int F, int k0, int k1) {
    return D > 0 && H > 0 && D % H == 0 && (D / H == 32 || D / H == 48) &&
           (D == 192 || D == 256 || D == 384) && F % 64 == 0 && (k0 * D) % 32 == 0 && (k1 * F) % 32 == 0 && (k0 & 1) &&
           (k1 & 1);
  };
  FL_REQUIRE(ok_stack(d[1], d[2], d[3], d[4], d[5]), "flamed_prior_create: unsupported encoder dims");
  FL_REQUIRE(ok_stack(d[8], d[9], d[10], d[11], d[12]), "flamed_prior_create: unsupported decoder dims");
  FL_REQUIRE(d[0] > 0 && d[6] >= 0 && d[7] > 0 && d[13] >= 0 && d[14] > 0 && d[15] > 0,
             "flamed_prior_create: bad symbol / layer / length / vocab dims");
  Prior* p = new Prior();
  p->n_sym = d[0];
  auto mk = [](int D, int H, int F, int k0, int k1, int nl, int maxseq) {
    FftStack s;
    s.D = D; s.H = H; s.F = F; s.k0 = k0; s.k1 = k1; s.maxseq = maxseq;
    s.layers.resize(nl);
    return s;
  };
  p->enc = mk(d[1], d[2], d[3], d[4], d[5], d[6], d[7]);
  p->shared = mk(d[8], d[9], d[10], d[11], d[12], d[13], d[14]);
  p->vocab = d[15];
  p->nq = nq;
  for (int q = 0; q < nq; ++q) p->dec.push_back(mk(d[8], d[9], d[10], d[11], d[12], d[17 + q], d[14]));
  p->head_n = (p->vocab + 1 + 63) / 64 * 64;
  *out = reinterpret_cast<flamed_prior_t>(p);
  return kOk;
}

FLAMED_API int flamed_prior_destroy(flamed_prior_t h) {
  Prior* p = reinterpret_cast<Prior*>(h);
  if (!p) return kOk;
  {
    std::lock_guard<std::mutex> lk(p->mu);
    DeviceGuard dg(p->device);
    p->genc.release();
    p->gdec.release();
    if (p->dev) (void)hipFree(p->dev);
    if (p->dev16) (void)hipFree(p->dev16);
    if (p->split_mem) (void)hipFree(p->split_mem);
  }
  delete p;
  return kOk;
}

FLAMED_API int flamed_prior_num_weights(flamed_prior_t h) {
  Prior* p = reinterpret_cast<Prior*>(h);
  return p ? n_weights(p) : -1;
}

FLAMED_API int flamed_prior_load(flamed_prior_t h, const float* const* w, int nw, hipStream_t st) {
  Prior* p = reinterpret_cast<Prior*>(h);
  FL_REQUIRE(p && w, "flamed_prior_load: null handle / weights");
  FL_REQUIRE(nw == n_weights(p), "flamed_prior_load: expected %d weights, got %d", n_weights(p), nw);
  for (int i = 0; i < nw; ++i) FL_REQUIRE(w[i], "flamed_prior_load: weight %d is null", i);
  int wdev = -1;
  FL_REQUIRE(device_of(w[0], &wdev) == kOk, "flamed_prior_load: weights must be device memory");
  for (int i = 1; i < nw; ++i) FL_REQUIRE_ON(w[i], wdev, "flamed_prior_load");
  std::lock_guard<std::mutex> lk(p->mu);
  if (p->device >= 0 && p->device != wdev) {
    DeviceGuard og(p->device);
    p->genc.release();
    p->gdec.release();
    if (p->dev) { (void)hipFree(p->dev); p->dev = nullptr; }
    if (p->dev16) { (void)hipFree(p->dev16); p->dev16 = nullptr; }
  }
  p->device = wdev;
  FL_ON_DEVICE(wdev);
  p->genc.release();
  p->gdec.release();
  if (p->dev) { FL_HIP(hipFree(p->dev)); p->dev = nullptr; }
  if (p->dev16) { FL_HIP(hipFree(p->dev16)); p->dev16 = nullptr; }  // stale copies: remade on the next bf16 decode

  // arena layout: packed items (qkv concat, conv taps, padded head) + plain copies (VecCopies)
  struct Pack { int kind; const float* src[3]; size_t n; int N, Cin, KT; const float** dst; size_t off; };
  std::vector<Pack> packs;
  VecCopies vc;
  size_t poff = 0;
  auto pack = [&](int kind, const float* a, const float* b, const float* c, size_t n, int N, int Cin, int KT, const float** dst) {
    packs.push_back(Pack{kind, {a, b, c}, n, N, Cin, KT, dst, poff});
    poff += a256(4 * n);
  };
  int i = 0;
  auto layers = [&](FftStack& s, int maxlen_rows) {
    vc.add(w[i++], (size_t)maxlen_rows * s.D, &s.pos);
    const size_t D = s.D, F = s.F;
    for (FftLayer& L : s.layers) {
      const float* const* lw = w + i;
      pack(0, lw[0], lw[2], lw[4], 3 * D * D, 0, 0, 0, &L.wqkv);      // w_qs / w_ks / w_vs weights
      pack(0, lw[1], lw[3], lw[5], 3 * D, 0, 0, 0, &L.bqkv);           // their biases
      vc.add(lw[6], D * D, &L.wfc); vc.add(lw[7], D, &L.bfc);
      vc.add(lw[8], D, &L.g1); vc.add(lw[9], D, &L.b1);
      pack(1, lw[10], nullptr, nullptr, F * s.k0 * D, (int)F, (int)D, s.k0, &L.w1);
      vc.add(lw[11], F, &L.c1b);
      pack(1, lw[12], nullptr, nullptr, D * s.k1 * F, (int)D, (int)F, s.k1, &L.w2);
      vc.add(lw[13], D, &L.c2b);
      vc.add(lw[14], D, &L.g2); vc.add(lw[15], D, &L.b2);
      i += kLayerW;
    }
  };
  const int De = p->enc.D, Dd = p->shared.D;
  vc.add(w[i++], (size_t)(p->n_sym + 1) * De, &p->src_emb);
  layers(p->enc, p->enc.maxseq + 1);
  vc.add(w[i++], (size_t)Dd * De, &p->bridge_w);
  vc.add(w[i++], Dd, &p->bridge_b);
  vc.add(w[i++], (size_t)(p->vocab + 1) * Dd, &p->code_emb);
  layers(p->shared, p->shared.maxseq + 1);
  vc.add(w[i++], Dd, &p->prompt_emb);
  vc.add(w[i++], Dd, &p->target_emb);
  vc.add(w[i++], (size_t)p->nq * Dd, &p->q_emb);
  for (FftStack& s : p->dec) layers(s, s.maxseq + 1);
  pack(2, w[i], nullptr, nullptr, (size_t)p->head_n * Dd, p->vocab + 1, Dd, 0, &p->head_w);
  pack(3, w[i + 1], nullptr, nullptr, (size_t)p->head_n, p->vocab + 1, 0, 0, &p->head_b);
  i += 2;
  FL_REQUIRE(i == nw, "flamed_prior_load: internal weight count mismatch (%d vs %d)", i, nw);

  const size_t total = a256(poff) + a256(vc.bytes);
  FL_HIP(hipMalloc(&p->dev, total));
  char* pb = p->dev;
  for (const Pack& k : packs) {
    float* dst = reinterpret_cast<float*>(pb + k.off);
    if (k.kind == 0) {  // concatenation of three equal parts
      const size_t part = k.n / 3;
      for (int j = 0; j < 3; ++j) FL_HIP(hipMemcpyAsync(dst + j * part, k.src[j], 4 * part, hipMemcpyDeviceToDevice, st));
    } else if (k.kind == 1) {  // conv taps-major
      hipLaunchKernelGGL(prior_taps_kernel, dim3((k.n + 255) / 256), dim3(256), 0, st, k.src[0], dst, k.N, k.Cin, k.KT);
      FL_LAUNCH_CHECK();
    } else {  // head weight / bias zero-padded to head_n rows
      const size_t valid = k.kind == 2 ? (size_t)k.N * k.Cin : (size_t)k.N;
      FL_HIP(hipMemsetAsync(dst, 0, 4 * k.n, st));
      FL_HIP(hipMemcpyAsync(dst, k.src[0], 4 * valid, hipMemcpyDeviceToDevice, st));
    }
    *k.dst = dst;
  }
  return vc.commit(pb + a256(poff), st);
}

FLAMED_API size_t flamed_prior_workspace_size(flamed_prior_t h, int B, int L, int T, int P) {
  Prior* p = reinterpret_cast<Prior*>(h);
  return p ? prior_ws_layout(p, B, L, T, P, nullptr, nullptr) : 0;
}

FLAMED_API int flamed_prior_encode(flamed_prior_t h, const int64_t* texts, const uint8_t* src_mask, int B, int L,
                                   const float* pos, float* out, void* ws, size_t ws_bytes, int use_graph, hipStream_t st) {
  Prior* p = reinterpret_cast<Prior*>(h);
  FL_REQUIRE(p && p->dev, "flamed_prior_encode: handle not loaded");
  FL_REQUIRE(texts && src_mask && out && ws && B > 0 && L > 0, "flamed_prior_encode: bad args");
  FL_REQUIRE(pos || L <= p->enc.maxseq, "flamed_prior_encode: L=%d exceeds the position table (%d): pass a table",
             L, p->enc.maxseq);
  std::lock_guard<std::mutex> lk(p->mu);
  FL_ON_DEVICE(p->device);
  FL_REQUIRE_ON(out, p->device, "flamed_prior_encode");
  const Tune tsnap = tune_snapshot(nullptr);
  TuneScope ts_(&tsnap);
  if (ws_bytes < prior_ws_layout(p, B, L, 0, 0, nullptr, nullptr)) {
    set_error("flamed_prior_encode: workspace too small");
    return kNoWorkspace;
  }
  PriorWs w;
  prior_ws_layout(p, B, L, 0, 0, ws, &w);
  std::vector<const void*> key = {texts, src_mask, pos, out, ws, (const void*)(intptr_t)B, (const void*)(intptr_t)L, p->dev};
  return with_graph(p->genc, key, use_graph != 0, st,
                    [&](hipStream_t s) { return run_encode(p, texts, src_mask, B, L, pos, out, w, s); });
}

FLAMED_API int flamed_prior_decode(flamed_prior_t h, const float* x, const uint8_t* tgt_mask, const int64_t* prompts, int B,
                                   int T, int P, const float* pos, float* embs, float* logits, void* ws, size_t ws_bytes,
                                   int use_graph, hipStream_t st) {
  Prior* p = reinterpret_cast<Prior*>(h);
  FL_REQUIRE(p && p->dev, "flamed_prior_decode: handle not loaded");
  FL_REQUIRE(x && tgt_mask && embs && logits && ws && B > 0 && T > 0 && P >= 0 && (P == 0 || prompts),
             "flamed_prior_decode: bad args");
  FL_REQUIRE(pos || P + T <= p->shared.maxseq, "flamed_prior_decode: P+T=%d exceeds the position table (%d): pass a table",
             P + T, p->shared.maxseq);
  std::lock_guard<std::mutex> lk(p->mu);
  FL_ON_DEVICE(p->device);
  FL_REQUIRE_ON(embs, p->device, "flamed_prior_decode");
  const Tune tsnap = tune_snapshot(nullptr);
  TuneScope ts_(&tsnap);
  if (ws_bytes < prior_ws_layout(p, B, 0, T, P, nullptr, nullptr)) {
    set_error("flamed_prior_decode: workspace too small");
    return kNoWorkspace;
  }
  PriorWs w;
  prior_ws_layout(p, B, 0, T, P, ws, &w);
  const bool b16 = p->dec_dt == FLAMED_BF16;
  if (b16 && !p->dev16) {
    int rc = ensure_bf16(p, st);
    if (rc) return rc;
  }
  std::vector<const void*> key = {x, tgt_mask, prompts, pos, embs, logits, ws, (const void*)(intptr_t)B,
                                  (const void*)(intptr_t)T, (const void*)(intptr_t)P, p->dev,
                                  (const void*)(intptr_t)p->dec_dt, p->dev16};
  return with_graph(p->gdec, key, use_graph != 0, st, [&](hipStream_t s) {
    if (!b16) return run_decode<float>(p, x, tgt_mask, prompts, B, T, P, pos, embs, logits, w, s);
    SplitScope sc(tn().prior_split ? &p->split : nullptr);
    return run_decode<bf16>(p, x, tgt_mask, prompts, B, T, P, pos, embs, logits, w, s);
  });
}

FLAMED_API int flamed_prior_set_dtype(flamed_prior_t h, int dtype) {
  Prior* p = reinterpret_cast<Prior*>(h);
  FL_REQUIRE(p, "flamed_prior_set_dtype: null handle");
  FL_REQUIRE(dtype == FLAMED_F32 || dtype == FLAMED_BF16, "flamed_prior_set_dtype: dtype must be FLAMED_F32 or FLAMED_BF16");
  std::lock_guard<std::mutex> lk(p->mu);
  p->dec_dt = dtype;
  return kOk;
}

}  // extern "C"
