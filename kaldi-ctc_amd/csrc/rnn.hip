// rnn.hip -- cuDNN-v5 compatible LSTM / GRU / RELU / TANH layers for gfx950.
//
// Replaces cudnnRNNForwardTraining / BackwardData / BackwardWeights as the
// reference calls them (src/cudamatrix/cudnn-recurrent.cc:13-102 through
// src/nnet2/nnet-cudnn-component.cc:508-614).  Per stacked layer:
//
// Forward
//   1. G = x W^T + bW (+ bR): the input projection of all T*N frames of both
//      directions as one packed split-fp16 GEMM (gemm_x3p.hip) -- or, for the
//      layers above the first, streamed off the previous component's running
//      recurrence (launch_chain_proj).
//   2. rnn_fwd_rec6: ONE persistent launch runs the whole time recurrence of
//      both directions (and of every row group of 8 or 16 sequences).  Work-
//      group (group, dir, g) owns hidden units [g*U, g*U+U); its slice of R
//      (nW*U gate rows x H) is held for the whole launch in REGISTERS as
//      split-fp16 MFMA B fragments (bf16 in configs[4]'s precision).  Per step
//      it loads h_{t-1} of its direction as fp16 hi/lo A fragments (sc1
//      buffer loads of the step's exchange image), multiplies on
//      v_mfma_f32_16x16x32_f16 (K split over the waves, reduced through LDS in
//      a fixed order), applies the gates (cell state in registers) and
//      publishes its U units of h_t as hi/lo fp16 with sc1 16-B stores.
// Backward data
//   rnn_bwd_rec6, reduce-scatter form: per step a workgroup sums the partial
//   dh of its own units from the direction's H/U producers (fixed order), adds
//   dy, does the pointwise cell backward (dc in registers), multiplies its
//   dGates by its R rows (registers) and publishes the partial dh of ALL H
//   units (MFMA C-fragment layout).  dGates rows go to the reserve, from where
//   the dx GEMM of the layer below is streamed while the recurrence runs
//   (x3p_bwd_stream_kernel).
// Backward weights
//   dW += dGx^T x, dR += dGh^T h_prev (time-shifted views), packed split-fp16
//   GEMMs on a side stream beside the next component's backward recurrence;
//   bias sums accumulated by the recurrence.
// Hand-off protocol (both recurrences): payload sc1 stores -> every storing
// wave's s_waitcnt vmcnt(0) -> workgroup barrier -> lane 0 stores the step
// epoch into the workgroup's own 128-B flag line; consumers poll the flag
// lines of their producers, then sc1 loads (MI355X_MICROARCH.md "Valid forms",
// row 1).  Every spin is bounded (3 s); a timeout sets the device error word,
// every workgroup drains out and the train step fails loudly.
// v4 (fp32 MFMA, XCD-slot all-gather) and v3 remain for the shapes v6 does
// not compile (RELU / TANH, other H, N > 64).
//
// Semantics follow cuDNN v5 as used by CuDNNRecurrentComponent: hx = cx = 0,
// dhy = dcy = 0 (SetBufferZero, nnet-cudnn-component.cc:494-506), all N
// sequences run the full T steps (no masking), weights in the opaque layout of
// nnet-cudnn-component.cc:327-413 (see RnnDesc::lin_offset).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "common.h"
#include "elementwise.h"
#include "gemm.h"
#include "prof.h"
#include "rnn.h"

#include <functional>

namespace kctc {

long RnnDesc::params_size() const {
  long t = 0;
  for (int l = 0; l < layers; l++) t += dirs * pl_size(l);
  return t;
}

long RnnDesc::lin_offset(int p, int lin, bool bias) const {
  long off = 0;
  for (int q = 0; q < p; q++) off += pl_size(q / dirs);
  const int layer = p / dirs, di = din(layer);
  const long n = nw();
  if (!bias) {
    if (lin < n) return off + (long)lin * H * di;
    return off + n * H * (long)di + (long)(lin - n) * H * H;
  }
  return off + n * H * (long)di + n * H * (long)H + (long)lin * H;
}

static long al64(long x) { return (x + 63) / 64 * 64; }
void rnn_set_precision(RnnDesc &d, int prec) {
  d.prec = prec;
  const char *e = getenv("KCTC_BF16_DIRECT");
  d.pk = !e || atoi(e) != 0;
  e = getenv("KCTC_BF16_IO");
  d.pkio = !e || atoi(e) != 0;
}

RnnReserveLayout rnn_reserve_layout(const RnnDesc &d, int T, int N) {
  RnnReserveLayout r;
  const long TN = (long)T * N, nw = d.nw(), H = d.H, dirs = d.dirs;
  long p = 0;
  r.G = p;    p += al64(TN * dirs * nw * H);
  r.aux = p;  p += al64(TN * dirs * H);
  r.E = p;    p += al64(TN * dirs * nw * H);
  r.DX = p;   p += (d.mode == kGru) ? al64(TN * dirs * nw * H) : 0;
  r.bias = p; p += al64(dirs * 2 * nw * H * (long)((N + 7) / 8));  // v6: per row group (>= 8 rows each)
  r.out = p;  p += (d.layers > 1) ? al64(TN * dirs * H) : 0;
  r.dout = p; p += (d.layers > 1) ? al64(TN * dirs * H) : 0;
  r.kbt64 = (TN + 63) / 64 * 64;
  const bool pkd = d.prec == 1 /* kPrecBf16 */ && d.layers == 1 && d.pk;  // bf16 halves: 2 per float
  const long G4 = nw * H, kbg64 = (G4 + 63) / 64 * 64;
  r.pkxr = p; p += pkd ? al64((dirs * TN * kbg64 + 1) / 2) : 0;
  r.pkxt = p; p += pkd ? al64((dirs * G4 * r.kbt64 + 1) / 2) : 0;
  const bool io = pkd && d.layers == 1 && dirs == 2;  // bf16_io: E^T shifted, apart from DX^T
  r.pket = p; p += (pkd && (d.mode == kGru || io)) ? al64((dirs * G4 * r.kbt64 + 1) / 2) : 0;
  r.pkyr = p; p += io ? al64((TN * dirs * H + 1) / 2) : 0;
  r.pkyc = p; p += io ? al64((dirs * H * r.kbt64 + 1) / 2) : 0;
  r.per_layer = p;
  r.total = p * d.layers;
  return r;
}

static long drec_split_floats(const RnnDesc &d, int T, int N) {
  // the dR and dW split slabs of a layer side by side: with a second stream
  // (rnn_backward_weights' s2) the two GEMMs run concurrently
  long need = 0, needR = 0, needW = 0;
  const int G4 = d.nw() * d.H;
  const int KB = (int)(((long)T * N + 31) / 32);  // packed k blocks over the frames (x3; bf16 needs fewer)
  for (int l = 0; l < d.layers; l++) {
    const long K = (long)(T > 1 ? T - 1 : 1) * N;
    int s = std::max(gemm_pick_split(G4, d.H, (int)K, d.dirs), x3p_pick_split(G4, d.H, KB, d.dirs));
    if (s > 1) needR = std::max(needR, (long)s * d.dirs * G4 * d.H);
    s = std::max(gemm_pick_split(G4, d.din(l), (int)((long)T * N), d.dirs), x3p_pick_split(G4, d.din(l), KB, d.dirs));
    if (s > 1) needW = std::max(needW, (long)s * d.dirs * G4 * d.din(l));
  }
  need = al64(needR) + needW;
  return need;
}

// split-K slabs of the weight-gradient GEMMs, then the recurrence flag words
static size_t flags_offset(const RnnDesc &d, int T, int N) {
  return sizeof(float) * (size_t)al64(drec_split_floats(d, T, N));
}
// then the v4 exchange images (one layer at a time; forward and backward of a
// layer never overlap): T * dirs * max(H, nW*H) * Npad floats
// flag region: words 0..1023 (v3/v4 flags, placement ids, GEMM tile counters
// at 1008/1009), then one 128-B line per (direction, workgroup) for v6
constexpr size_t kFlagBytes = 4096 + 512 * 128;  // v6: up to 4 row groups x 2 dirs x 64 workgroups
static size_t xch_offset(const RnnDesc &d, int T, int N) { return flags_offset(d, T, N) + kFlagBytes; }
static size_t xch_bytes(const RnnDesc &d, int T, int N) {
  const long Npad = (N + 15) / 16 * 16;
  // v4 images: 4 B x dirs x nW x H x Npad per step; the v6 forward's
  // [2 dirs][H/32][hi, lo][16][32] halves per row group of <= 16 rows (at most
  // 2 Npad / 16 groups): 16 B x H x Npad.  + 2 steps: the v6 forward's ring of
  // hand-off images after its T step images
  const size_t per = std::max<size_t>(sizeof(float) * d.dirs * d.nw(), 16);
  return per * (size_t)(T + 2) * d.H * Npad;
}
// then the packed split-fp16 GEMM operands of one layer at a time (forward,
// backward-data and the weight GEMMs of a component never overlap):
//   forward   : input rows [TN][Din], W rows [dirs*G][Din]
//   bwd data  : dGates rows [dirs*TN][G], W^T rows [dirs*Din][G]
//   bwd weight: dGates^T [dirs*G][TN] (+ GRU: E^T), input^T [Din][TN],
//               shifted output^T [dirs*H][TN]
// plus int exponents and float-bit column maxima (G = nW*H).
struct PackLay {
  size_t a, b, c, d, ea, eb, ec, ed, cm, part, cnt, part2, cme, fcnt, fpart, wt, ewt, cmw, xt, yt, ext, eyt, pcnt, total;
};
static PackLay pack_layout(const RnnDesc &d, int T, int N) {
  const long TN = (long)T * N, G = (long)d.nw() * d.H, Dm = std::max(d.D, d.dirs * d.H), dirs = d.dirs;
  const size_t fw_a = x3p_bytes(TN, Dm), fw_b = x3p_bytes(dirs * G, Dm);
  const size_t bd_a = x3p_bytes(dirs * TN, G), bd_b = x3p_bytes(dirs * Dm, G);
  const size_t bw_a = x3p_bytes(dirs * G, TN) * (d.mode == kGru ? 2 : 1), bw_b = x3p_bytes(Dm, TN),
               bw_c = x3p_bytes(dirs * d.H, TN);
  PackLay p;
  size_t o = 0;
  p.a = o; o = align_up(o + std::max({fw_a, bd_a, bw_a}), 256);
  p.b = o; o = align_up(o + std::max({fw_b, bd_b, bw_b}), 256);
  p.c = o; o = align_up(o + bw_c, 256);
  p.d = o;  // unused slot kept for symmetry (0 bytes)
  const long ne = std::max({TN * dirs, dirs * G * 2, dirs * Dm}) + 64;
  p.ea = o; o = align_up(o + sizeof(int) * ne, 256);
  p.eb = o; o = align_up(o + sizeof(int) * ne, 256);
  p.ec = o; o = align_up(o + sizeof(int) * ne, 256);
  p.ed = o; o = align_up(o + sizeof(int) * ne, 256);
  p.cm = o; o = align_up(o + sizeof(unsigned) * ne, 256);
  p.part = o; o = align_up(o + sizeof(float) * x3p_bwd_stream_part_floats((int)TN, (int)Dm), 256);  // backward stream partials
  // (also the row stream of this component's projection off the previous
  // component's forward, launch_chain_rows: N = dirs * G columns)
  p.cnt = o; o = align_up(o + sizeof(int) * x3p_bwd_stream_ints((int)TN, (int)std::max(Dm, dirs * G)), 256);
  p.part2 = o; o = align_up(o + sizeof(float) * x3p_bwd_stream_part2_floats((int)std::max(Dm, dirs * G)), 256);
  p.cme = o; o = align_up(o + sizeof(unsigned) * 2 * dirs * G, 256);  // dGates column maxima (v6 backward)
  // arrival counters of the direction-split streamed projection (this component as its consumer)
  p.fcnt = o; o = align_up(o + sizeof(int) * ((TN + 127) / 128 * dirs * ((G + 127) / 128) + 64), 256);
  p.fpart = o; o = align_up(o + sizeof(float) * std::max((size_t)((TN + 127) / 128) * dirs * ((G + 127) / 128) * 128 * 128,
                                                          x3p_bwd_stream_part_floats((int)TN, (int)(dirs * G))), 256);
  // W^T of the streamed dx GEMM, packed by the forward (RnnPrepack): kept
  // from the forward to the backward, apart from every other slot
  p.wt = o; o = align_up(o + x3p_bytes(dirs * Dm, G), 256);
  p.ewt = o; o = align_up(o + sizeof(int) * (dirs * Dm + 64), 256);
  p.cmw = o; o = align_up(o + sizeof(unsigned) * (dirs * Dm + 64), 256);
  // x^T / y^T of the weight GEMMs, packed by the forward (RnnPrepack::wgrad)
  p.xt = o; o = align_up(o + bw_b, 256);
  p.yt = o; o = align_up(o + bw_c, 256);
  p.ext = o; o = align_up(o + sizeof(int) * (Dm + 64), 256);
  p.eyt = o; o = align_up(o + sizeof(int) * (dirs * d.H + 64), 256);
  // item counters of those packs (on the prepack stream; apart from the
  // recurrence flags, which the backward resets on the compute stream)
  p.pcnt = o; o = align_up(o + sizeof(int) * 4, 256);
  p.total = o;
  return p;
}
static size_t pack_offset(const RnnDesc &d, int T, int N) { return align_up(xch_offset(d, T, N) + xch_bytes(d, T, N), 256); }
size_t rnn_workspace_bytes(const RnnDesc &d, int T, int N) { return pack_offset(d, T, N) + pack_layout(d, T, N).total; }
template <typename P>
static P *pk(void *ws, const RnnDesc &d, int T, int N, size_t off) {
  return reinterpret_cast<P *>(static_cast<char *>(ws) + pack_offset(d, T, N) + off);
}
// The RNN GEMMs run on the packed split-fp16 matrix-core path (gemm_x3p.hip)
// unless the contraction is too short to pay for packing.
static bool use_x3(int K, int min_k = 128) {
  return K >= min_k;
}
// |x| <= 1: an LSTM / GRU / TANH layer output
static bool bounded_out(const RnnDesc &d) { return d.mode != kRelu; }

namespace {
int env_int(const char *name, int dflt);
}  // namespace

// bf16 recurrences write their dGates straight into the packed bf16 GEMM
// operands (RecParams::dxr / dxt / et) -- v6 only (a v6 backward runs for
// every bf16 shape), whole 64-element gate rows
// (one-layer descriptors -- the recipe's components; a stacked descriptor's
// weight gradients measured wrong with it, so those keep the pack path)
static bool bf16_direct(const RnnDesc &d, int ver) {
  return d.prec == 1 /* kPrecBf16 */ && ver == 6 && (d.nw() * d.H) % 64 == 0 && d.layers == 1 && d.pk;
}
// ... and, one-layer bidirectional, the forward writes its output packed
// (RecParams::yr / yc) and the backward E^T shifted (eshift); H % 32 == 0 so
// that a workgroup's units fill whole 16-B row chunks
static bool bf16_io(const RnnDesc &d) {
  return bf16_direct(d, 6) && d.layers == 1 && d.dirs == 2 && d.H % 32 == 0 && (2 * d.H) % 64 == 0 && d.pkio;
}



namespace {

constexpr int NT = 256;
constexpr unsigned kSent = 0xFFFFFFFFu;
constexpr int kSpinLimit = 1 << 21;
constexpr int kMaxRT = 4;  // N <= 64 (four 16-row MFMA tiles)
constexpr int kMaxCT = 4;  // <= 64 gate columns per workgroup

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bool ready4(u32x4 v) {
  return (v[0] != kSent) & (v[1] != kSent) & (v[2] != kSent) & (v[3] != kSent);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, bytes, 0x00020000);
}

__device__ __forceinline__ u32x4 ld_sc1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16 /* sc1 */);
}

// Re-poll one 16-byte fragment until it holds no sentinel (bounded spin).
__device__ __forceinline__ u32x4 settle(__amdgpu_buffer_rsrc_t r, unsigned off, u32x4 v,
                                        unsigned *err, int &bad) {
  int spins = 0;
  while (!bad && !ready4(v)) {
    if (++spins > kSpinLimit) { bad = 1; break; }
    if ((spins & 255) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
      bad = 1;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
    v = ld_sc1(r, off);
  }
  return v;
}

__device__ __forceinline__ void publish(float *p, float v) {
  unsigned u = __float_as_uint(v);
  if (u == kSent) u = 0x7FC00000u;  // never publish the sentinel bit pattern
  __hip_atomic_store(reinterpret_cast<unsigned *>(p), u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

struct RecParams {
  int T, N, H, dirs, U, nwg, ncol, Npad;
  int rg;           // v6: row groups (independent recurrences) of gs sequences
  int gs;           // v6: sequences per row group (16, or 8: two groups of a 16-row batch run side by side)
  const float *w;   // params base of this stacked layer's pseudo-layer 0
  long pl_stride;   // floats between the two directions' blocks
  long r_off;       // R within a pseudo-layer block
  long bR_off;      // bR within a pseudo-layer block
  float *G;         // [T*N][dirs*nW*H] pre-activations -> activations
  float *y;         // [T*N][dirs*H] output / h exchange (sentinel pre-filled)
  float *aux;       // LSTM: c ; GRU: R_n h + b_Rn   [T*N][dirs*H]
  const float *dy;  // backward: [T*N][dirs*H]
  float *E;         // backward: dGates (recurrent part) exchange [T*N][dirs*nW*H]
  float *DX;        // backward GRU: dGates (input part); == E otherwise
  float *bias;      // backward: bias partial sums [dirs][2][nW*H]
  unsigned *flags;  // flag protocol: [dirs][nwg] step epochs, zeroed before launch
  unsigned *err;
  int sync;         // kSyncData / kSyncFlag
  unsigned long long *trace;  // optional: [kTraceSteps][grid][8] s_memrealtime stamps
  int allow_local;  // v4: hand off through the shared L2 when placement allows it
  int xpd;          // v4: XCD slots per direction (nwg = 32 * xpd workgroups)
  int ring;         // v6: hand-off images reused every `ring` steps (0: one image per step; forward: ring after the T step images)
  int fcopy;        // v6 forward, XCD-pinned: h images also written through (sc1) per step for a streamed projection
  float *xch;       // v4: per-step exchange images [T][dirs][KG][Npad][16] (workspace)
  int poll_sleep;   // v6: s_sleep between flag polls
  int gla;          // v6 forward IO waves: steps ahead the G rows are fetched (3 or 7; 8 LDS slots)
  int e_sc1;        // v6 backward: dGates rows written through (sc1) for a streaming consumer
  int ysc1;         // v6 forward: y rows written through (sc1) and the aggregated epochs published
                    // for the next component's projection streamed off them (launch_chain_rows)
  int bfpart;       // v6 backward, bf16 mode: partial dh exchanged as bf16
  unsigned *cmax;   // v6 backward: column max |DX| [dirs * nW * H] (GRU: then |E|), as float bits
  unsigned *reg;    // v6 backward: per-device registration word (+1 per workgroup at start)
  // v6 backward, bf16 (RnnReserveLayout::pk): dGates written straight into the
  // packed bf16 operands of the GEMMs after the recurrence, instead of fp32
  // rows that pack kernels re-read: dxr = DX rows [dir][T*N][nW*H] (A of the
  // dx GEMM), dxt = DX^T [dir][nW*H][kbt64] (A of dW), et = E^T (A of dR; ==
  // dxt for an LSTM), frames along the packed rows (kbt64 >= T*N, zero tail)
  __bf16 *dxr, *dxt, *et;
  long kbt64;
  // bf16 one-layer bidirectional (bf16_io): the forward writes its output h as
  // packed bf16 too -- yr = rows [T*N][dirs*H] (A of the next component's
  // input projection), yc = columns [dirs*H][kbt64] (B of this component's dR
  // and of the next component's dW) -- and the backward then writes E^T
  // shifted by one step (eshift: direction 0 frame f at f - N, direction 1 at
  // f + N), so that dR pairs it with the unshifted yc
  __bf16 *yr, *yc;
  int eshift;
  // v6 backward, fp32 partials, ring of 2: self-tagged hand-off (see
  // rnn_bwd_rec6): the consumers poll the partial-dh words themselves instead
  // of the producers' epoch flags; taken by the slots probe6 finds XCD-local
  // (v6 forward, split-fp16 without IO waves: the same for the h hi / lo
  // halves, each carrying the tag in its LSB)
  int dtag;
};

// Phase stamps of the first kTraceSteps steps ([steps][grid][16]; thread 0 of every workgroup;
// 100 MHz constant clock), only when the host passes a trace buffer
// (KCTC_REC_TRACE): 0 step start, 1 flags seen, 2 operand loads landed,
// 3 MFMA + K reduction done, 4 published (+ flag), 5 step end.
// v6 backward: slots 16 + w flags seen by wave w, 24 + w its hand-off loads landed.
constexpr int kTraceSteps = 256, kTraceStride = 32;
// (the cursor trc_ / trg_ of REC_TRACE_INIT lives in VGPRs: the stamps cost
// the step loop no scalar registers)
#define REC_TRACE_INIT                                                                    \
  unsigned long long *trc_ = p.trace ? p.trace + (long)blockIdx.x * kTraceStride : nullptr; \
  long trg_ = (long)gridDim.x * kTraceStride;                                             \
  asm volatile("" : "+v"(trc_), "+v"(trg_))
#define REC_TRACE(kk, ph)                                                                 \
  do {                                                                                    \
    if (trc_ && threadIdx.x == 0 && (kk) < kTraceSteps) {                                 \
      unsigned long long *tr_ = trc_ + (long)(kk) * trg_;                                 \
      tr_[(ph)] = __builtin_amdgcn_s_memrealtime();                                       \
      if ((ph) == 2 || (ph) == 3) tr_[12 + (ph)] = __builtin_amdgcn_s_memtime();          \
    }                                                                                     \
  } while (0)
// per-wave stamps (lane 0 of every wave): slot 6 + w loads landed, 10 + w MFMA done;
// slots 14/15: shader-clock counter (s_memtime) at phases 2/3 (clock estimate)
#define REC_TRACE_W(kk, ph)                                                               \
  do {                                                                                    \
    if (trc_ && (threadIdx.x & 63) == 0 && (kk) < kTraceSteps)                            \
      trc_[(long)(kk) * trg_ + (ph) + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

// Hand-off protocols (selected per launch; both placement-independent):
//  kSyncData: the payload is the flag (sentinel-filled buffer, sc1 4-B stores,
//             sc1 16-B loads re-polled until no sentinel is left).
//  kSyncFlag: payload sc1 stores -> every storing wave s_waitcnt vmcnt(0) ->
//             workgroup barrier -> ONE lane stores the step epoch (sc1) into
//             the workgroup's flag word; consumers: wave 0 polls the nwg flag
//             words of its direction with one sc1 load per lane, barrier, then
//             every wave loads the payload with sc1 loads (MI355X_MICROARCH.md
//             "Valid forms", row 1).  Polling traffic: 4 B per producer, not
//             the whole payload.
enum { kSyncData = 0, kSyncFlag = 1 };

__device__ __forceinline__ void wait_flags(const unsigned *flags, int nwg, unsigned epoch,
                                           unsigned *err, int &bad, int *bad_lds) {
  if (threadIdx.x < 64) {
    int spins = 0;
    while (true) {
      bool ok = true;
      for (int i = threadIdx.x; i < nwg; i += 64)
        ok &= __hip_atomic_load(flags + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= epoch;
      if (__all(ok)) break;
      if (++spins > kSpinLimit ||
          ((spins & 255) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        bad = 1;
        if (threadIdx.x == 0) *bad_lds = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (*bad_lds) bad = 1;
}

__device__ __forceinline__ void signal_flag(unsigned *flag, unsigned epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A-operand fragments of one step: rows n (RT 16-row tiles) x this wave's
// k-groups {w, w+4, ...}, CH k-groups per pass, straight from the exchange
// buffer into registers with sc1 16-B loads.  Returns false on timeout.
template <int RT, int CH>
__device__ __forceinline__ void load_frags(u32x4 (&af)[RT][CH], __amdgpu_buffer_rsrc_t rs, long ld,
                                           long col0, int c0, int KG, int N, int sync, unsigned *err,
                                           int &bad) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int i = 0; i < CH; i++) {
    const int kg = w + 4 * (c0 + i);
#pragma unroll
    for (int rt = 0; rt < RT; rt++) {
      const int n = rt * 16 + fr;
      af[rt][i] = u32x4{0u, 0u, 0u, 0u};
      if (kg < KG && n < N) af[rt][i] = ld_sc1(rs, (unsigned)(((long)n * ld + col0 + kg * 16 + fq * 4) * 4));
    }
  }
  if (sync == kSyncData) {
#pragma unroll
    for (int i = 0; i < CH; i++) {
      const int kg = w + 4 * (c0 + i);
#pragma unroll
      for (int rt = 0; rt < RT; rt++) {
        const int n = rt * 16 + fr;
        if (kg < KG && n < N)
          af[rt][i] = settle(rs, (unsigned)(((long)n * ld + col0 + kg * 16 + fq * 4) * 4), af[rt][i], err, bad);
      }
    }
  }
}

// 16-byte write-through (sc1) publish of 4 consecutive units: every A-operand
// fragment a consumer loads (4 consecutive k) is exactly one such store, so a
// fragment is either all-sentinel or all-final (no tearing to re-poll).
__device__ __forceinline__ floatx4 canon(floatx4 v) {
#pragma unroll
  for (int i = 0; i < 4; i++)
    if (__float_as_uint(v[i]) == kSent) v[i] = __uint_as_float(0x7FC00000u);
  return v;
}
__device__ __forceinline__ void publish4(__amdgpu_buffer_rsrc_t r, unsigned off, floatx4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, canon(v)), r, (int)off, 0, 16);
}
__device__ __forceinline__ floatx4 ld4(const float *p) { return *reinterpret_cast<const floatx4 *>(p); }
__device__ __forceinline__ void st4(float *p, floatx4 v) { *reinterpret_cast<floatx4 *>(p) = v; }
__device__ __forceinline__ floatx4 sigm4(floatx4 x) {
  floatx4 r;
#pragma unroll
  for (int i = 0; i < 4; i++) r[i] = sigm(x[i]);
  return r;
}
__device__ __forceinline__ floatx4 tanh4(floatx4 x) {
  floatx4 r;
#pragma unroll
  for (int i = 0; i < 4; i++) r[i] = tanhf(x[i]);
  return r;
}

// Poll every not-yet-valid fragment of this lane in batches: all re-loads of
// a round are in flight together, so a round costs one memory round trip.
template <int RT, int CH>
__device__ __forceinline__ void settle_all(u32x4 (&af)[RT][CH], __amdgpu_buffer_rsrc_t rs, long ld,
                                           long col0, int c0, int KG, int N, unsigned *err, int &bad) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fq = lane >> 4;
  for (int round = 0; !bad; round++) {
    int pending = 0;
#pragma unroll
    for (int i = 0; i < CH; i++) {
      const int kg = w + 4 * (c0 + i);
#pragma unroll
      for (int rt = 0; rt < RT; rt++) {
        const int n = rt * 16 + fr;
        if (kg < KG && n < N && !ready4(af[rt][i])) {
          af[rt][i] = ld_sc1(rs, (unsigned)(((long)n * ld + col0 + kg * 16 + fq * 4) * 4));
          pending++;
        }
      }
    }
    if (!pending) break;
    if (round > kSpinLimit ||
        ((round & 255) == 255 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
      bad = 1;
      break;
    }
    asm volatile("" ::: "memory");
  }
}

// ---------------------------------------------------------------------------
// forward recurrence
// ---------------------------------------------------------------------------
template <int MODE, int RT>
__global__ __launch_bounds__(NT, 1) void rnn_fwd_rec(RecParams p) {
  REC_TRACE_INIT;
  constexpr int NW = MODE == kLstm ? 4 : MODE == kGru ? 3 : 1;
  constexpr int CH = 32 / RT;  // k-groups per wave per pass (<= 32 A-fragment registers x4)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int bad_lds;
  const int H = p.H, U = p.U, N = p.N, T = p.T, ncol = p.ncol;
  const int LDR = H + 4;
  const int d = blockIdx.x / p.nwg, g = blockIdx.x % p.nwg, u0 = g * U;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int CT = ncol / 16;
  const long ldy = (long)p.dirs * H, ldg = (long)p.dirs * NW * H;
  float *Rs = smem;                      // [ncol][LDR]
  float *red = Rs + (long)ncol * LDR;    // [4][Npad][ncol]
  const float *Wd = p.w + d * p.pl_stride;
  const float *R = Wd + p.r_off;
  if (tid == 0) bad_lds = 0;
  for (int idx = tid; idx < ncol * H; idx += NT) {
    const int c = idx / H, k = idx - c * H;
    float v = 0.f;
    if (c < NW * U) {
      const int gt = c / U, u = c - gt * U;
      v = R[(long)(gt * H + u0 + u) * H + k];
    }
    Rs[c * LDR + k] = v;
  }
  // pointwise item of this thread: row n, units u0+4q .. u0+4q+3
  const int Q = U / 4, items = N * Q;
  const bool has_item = tid < items;
  const int in_ = has_item ? tid / Q : 0, iq = has_item ? tid - in_ * Q : 0;
  const int ucol = u0 + 4 * iq;
  floatx4 cst = {0.f, 0.f, 0.f, 0.f}, hpv = cst, gin[NW], bR[NW];
#pragma unroll
  for (int q = 0; q < NW; q++) {
    bR[q] = (MODE == kGru && has_item) ? ld4(Wd + p.bR_off + q * H + ucol) : floatx4{0.f, 0.f, 0.f, 0.f};
    gin[q] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  if (has_item) {  // prefetch the input projection of the first step
    const int t = d == 0 ? 0 : T - 1;
#pragma unroll
    for (int q = 0; q < NW; q++) gin[q] = ld4(p.G + ((long)t * N + in_) * ldg + (long)d * NW * H + q * H + ucol);
  }
  __syncthreads();
  int bad = 0;
  const int KG = H / 16;
  const int KGW = (KG + 3) / 4;  // k-groups per wave
  const unsigned step_bytes = (unsigned)((long)N * ldy * sizeof(float));
  unsigned *myflag = p.flags + d * p.nwg + g;
  for (int k = 0; k < T; k++) {
    const int t = d == 0 ? k : T - 1 - k, tp = d == 0 ? t - 1 : t + 1;
    floatx4 acc[RT][kMaxCT];
#pragma unroll
    for (int a = 0; a < RT; a++)
#pragma unroll
      for (int b = 0; b < kMaxCT; b++) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    REC_TRACE(k, 0);
    if (k > 0) {
      if (p.sync == kSyncFlag) wait_flags(p.flags + d * p.nwg, p.nwg, (unsigned)k, p.err, bad, &bad_lds);
      REC_TRACE(k, 1);
      const auto rs = rsrc(p.y + (long)tp * N * ldy, step_bytes);
      for (int c0 = 0; c0 < KGW; c0 += CH) {
        u32x4 af[RT][CH];
        load_frags<RT, CH>(af, rs, ldy, (long)d * H, c0, KG, N, kSyncFlag, p.err, bad);
        if (p.sync == kSyncData) settle_all<RT, CH>(af, rs, ldy, (long)d * H, c0, KG, N, p.err, bad);
        if (p.trace) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          REC_TRACE(k, 2);
        }
#pragma unroll
        for (int i = 0; i < CH; i++) {
          const int kg = w + 4 * (c0 + i);
          if (kg < KG) {
#pragma unroll
            for (int ct = 0; ct < kMaxCT; ct++) {
              if (ct < CT) {
                const floatx4 b = ld4(Rs + (ct * 16 + fr) * LDR + kg * 16 + fq * 4);
#pragma unroll
                for (int s = 0; s < 4; s++)
#pragma unroll
                  for (int rt = 0; rt < RT; rt++)
                    acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[rt][i][s]), b[s],
                                                                       acc[rt][ct], 0, 0, 0);
              }
            }
          }
        }
      }
    }
    // cross-wave K reduction through LDS
#pragma unroll
    for (int rt = 0; rt < RT; rt++)
#pragma unroll
      for (int ct = 0; ct < kMaxCT; ct++)
        if (ct < CT)
#pragma unroll
          for (int r = 0; r < 4; r++)
            red[((long)w * p.Npad + rt * 16 + fq * 4 + r) * ncol + ct * 16 + fr] = acc[rt][ct][r];
    __syncthreads();
    REC_TRACE(k, 3);
    floatx4 act[NW], cnew = {0.f, 0.f, 0.f, 0.f};
    const long yrow = ((long)t * N + in_) * ldy + (long)d * H + ucol;
    if (has_item) {
      floatx4 rh[NW];
#pragma unroll
      for (int q = 0; q < NW; q++) {
        const int c = q * U + 4 * iq;
        rh[q] = ((ld4(red + ((long)0 * p.Npad + in_) * ncol + c) + ld4(red + ((long)1 * p.Npad + in_) * ncol + c)) +
                 ld4(red + ((long)2 * p.Npad + in_) * ncol + c)) + ld4(red + ((long)3 * p.Npad + in_) * ncol + c);
      }
      floatx4 h;
      if (MODE == kLstm) {
        act[0] = sigm4(gin[0] + rh[0]);
        act[1] = sigm4(gin[1] + rh[1]);
        act[2] = tanh4(gin[2] + rh[2]);
        act[3] = sigm4(gin[3] + rh[3]);
        cst = act[1] * cst + act[0] * act[2];
        cnew = cst;
        h = act[3] * tanh4(cst);
      } else if (MODE == kGru) {
        act[0] = sigm4(gin[0] + rh[0] + bR[0]);
        act[1] = sigm4(gin[1] + rh[1] + bR[1]);
        cnew = rh[2] + bR[2];
        act[2] = tanh4(gin[2] + act[0] * cnew);
        h = (1.f - act[1]) * act[2] + act[1] * hpv;
        hpv = h;
      } else {
        const floatx4 pre = gin[0] + rh[0];
        if (MODE == kRelu) {
#pragma unroll
          for (int i = 0; i < 4; i++) h[i] = fmaxf(pre[i], 0.f);
        } else {
          h = tanh4(pre);
        }
      }
      publish4(rsrc(p.y + (long)t * N * ldy, step_bytes), (unsigned)(((long)in_ * ldy + (long)d * H + ucol) * 4), h);
    }
    if (p.sync == kSyncFlag) signal_flag(myflag, (unsigned)(k + 1));
    REC_TRACE(k, 4);
    if (has_item) {
      const long grow = ((long)t * N + in_) * ldg + (long)d * NW * H + ucol;
      if (MODE == kLstm || MODE == kGru) {
#pragma unroll
        for (int q = 0; q < NW; q++) st4(p.G + grow + q * H, act[q]);
        st4(p.aux + yrow, cnew);
      }
      if (k + 1 < T) {  // prefetch the next step's input projection
        const int tn = d == 0 ? t + 1 : t - 1;
#pragma unroll
        for (int q = 0; q < NW; q++) gin[q] = ld4(p.G + ((long)tn * N + in_) * ldg + (long)d * NW * H + q * H + ucol);
      }
    }
    __syncthreads();  // red[] is rewritten by the next step
    REC_TRACE(k, 5);
  }
  if (bad && tid == 0) atomicOr(p.err, 1u);
}

// ---------------------------------------------------------------------------
// backward-data recurrence
// ---------------------------------------------------------------------------
template <int MODE, int RT>
__global__ __launch_bounds__(NT, 1) void rnn_bwd_rec(RecParams p) {
  REC_TRACE_INIT;
  constexpr int NW = MODE == kLstm ? 4 : MODE == kGru ? 3 : 1;
  constexpr int CH = 32 / RT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int bad_lds;
  const int H = p.H, U = p.U, N = p.N, T = p.T;
  const int K = NW * H, LDK = K + 4;
  const int d = blockIdx.x / p.nwg, g = blockIdx.x % p.nwg, u0 = g * U;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const long ldy = (long)p.dirs * H, ldg = (long)p.dirs * NW * H;
  float *RT_s = smem;                       // [U][LDK]: RT_s[u][kk] = R[kk][u0+u]
  float *red = RT_s + (long)U * LDK;        // [4][Npad][16]
  const float *Wd = p.w + d * p.pl_stride;
  const float *R = Wd + p.r_off;
  if (tid == 0) bad_lds = 0;
  for (int idx = tid; idx < U * K; idx += NT) {
    const int kk = idx / U, u = idx - kk * U;
    RT_s[u * LDK + kk] = R[(long)kk * H + u0 + u];
  }
  const int Q = U / 4, items = N * Q;
  const bool has_item = tid < items;
  const int in_ = has_item ? tid / Q : 0, iq = has_item ? tid - in_ * Q : 0;
  const int ucol = u0 + 4 * iq;
  const floatx4 z4 = {0.f, 0.f, 0.f, 0.f};
  floatx4 carry = z4;  // LSTM: dc carried to the previous step; GRU: dh*z direct term
  floatx4 bsx[NW], bsh[NW], pg[NW], pdy = z4, pa = z4, pap = z4;
#pragma unroll
  for (int q = 0; q < NW; q++) bsx[q] = bsh[q] = pg[q] = z4;
  auto prefetch = [&](int k) {
    if (!has_item) return;
    const int t = d == 0 ? k : T - 1 - k, tp = d == 0 ? t - 1 : t + 1;
    const long yrow = ((long)t * N + in_) * ldy + (long)d * H + ucol;
    const long grow = ((long)t * N + in_) * ldg + (long)d * NW * H + ucol;
    const long prow = ((long)tp * N + in_) * ldy + (long)d * H + ucol;
    pdy = ld4(p.dy + yrow);
    if (MODE == kLstm || MODE == kGru) {
#pragma unroll
      for (int q = 0; q < NW; q++) pg[q] = ld4(p.G + grow + q * H);
      pa = ld4(p.aux + yrow);
    }
    if (MODE == kLstm) pap = k > 0 ? ld4(p.aux + prow) : z4;
    else if (MODE == kGru) pap = k > 0 ? ld4(p.y + prow) : z4;
    else pap = ld4(p.y + yrow);
  };
  prefetch(T - 1);
  __syncthreads();
  int bad = 0;
  const int KG = K / 16;
  const int KGW = (KG + 3) / 4;
  const unsigned step_bytes = (unsigned)((long)N * ldg * sizeof(float));
  unsigned *myflag = p.flags + d * p.nwg + g;
  for (int k = T - 1; k >= 0; k--) {
    const int t = d == 0 ? k : T - 1 - k;       // forward-order index k
    const int tn = d == 0 ? t + 1 : t - 1;      // processed just before (k+1)
    const unsigned epoch = (unsigned)(T - k);   // number of steps published so far
    floatx4 acc[RT];
#pragma unroll
    for (int a = 0; a < RT; a++) acc[a] = z4;
    const int ks = T - 1 - k;
    REC_TRACE(ks, 0);
    if (k < T - 1) {
      if (p.sync == kSyncFlag) wait_flags(p.flags + d * p.nwg, p.nwg, epoch - 1, p.err, bad, &bad_lds);
      REC_TRACE(ks, 1);
      const auto rs = rsrc(p.E + (long)tn * N * ldg, step_bytes);
      for (int c0 = 0; c0 < KGW; c0 += CH) {
        u32x4 af[RT][CH];
        load_frags<RT, CH>(af, rs, ldg, (long)d * K, c0, KG, N, kSyncFlag, p.err, bad);
        if (p.sync == kSyncData) settle_all<RT, CH>(af, rs, ldg, (long)d * K, c0, KG, N, p.err, bad);
        if (p.trace) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          REC_TRACE(ks, 2);
        }
#pragma unroll
        for (int i = 0; i < CH; i++) {
          const int kg = w + 4 * (c0 + i);
          if (kg < KG) {
            floatx4 b = z4;
            if (fr < U) b = ld4(RT_s + fr * LDK + kg * 16 + fq * 4);
#pragma unroll
            for (int s = 0; s < 4; s++)
#pragma unroll
              for (int rt = 0; rt < RT; rt++)
                acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[rt][i][s]), b[s], acc[rt], 0, 0, 0);
          }
        }
      }
    }
#pragma unroll
    for (int rt = 0; rt < RT; rt++)
#pragma unroll
      for (int r = 0; r < 4; r++) red[((long)w * p.Npad + rt * 16 + fq * 4 + r) * 16 + fr] = acc[rt][r];
    __syncthreads();
    REC_TRACE(ks, 3);
    floatx4 dxk[NW];
    const long grow = ((long)t * N + in_) * ldg + (long)d * NW * H + ucol;
    const auto rsE = rsrc(p.E + (long)t * N * ldg, step_bytes);
    const unsigned eoff = (unsigned)(((long)in_ * ldg + (long)d * NW * H + ucol) * 4);
    if (has_item) {
      const floatx4 dhr = ((ld4(red + ((long)0 * p.Npad + in_) * 16 + 4 * iq) + ld4(red + ((long)1 * p.Npad + in_) * 16 + 4 * iq)) +
                           ld4(red + ((long)2 * p.Npad + in_) * 16 + 4 * iq)) + ld4(red + ((long)3 * p.Npad + in_) * 16 + 4 * iq);
      floatx4 dh = pdy + dhr;
      if (MODE == kLstm) {
        const floatx4 ig = pg[0], fg = pg[1], gg = pg[2], og = pg[3];
        const floatx4 tc = tanh4(pa);
        const floatx4 dO = dh * tc;
        const floatx4 dc = dh * og * (1.f - tc * tc) + carry;
        const floatx4 dpi = dc * gg * ig * (1.f - ig);
        const floatx4 dpf = dc * pap * fg * (1.f - fg);
        const floatx4 dpg = dc * ig * (1.f - gg * gg);
        const floatx4 dpo = dO * og * (1.f - og);
        carry = dc * fg;
        publish4(rsE, eoff, dpi);
        publish4(rsE, eoff + 4 * H, dpf);
        publish4(rsE, eoff + 8 * H, dpg);
        publish4(rsE, eoff + 12 * H, dpo);
        bsx[0] += dpi; bsx[1] += dpf; bsx[2] += dpg; bsx[3] += dpo;
      } else if (MODE == kGru) {
        dh += carry;
        const floatx4 r = pg[0], z = pg[1], nn = pg[2];
        const floatx4 dn = dh * (1.f - z), dz = dh * (pap - nn);
        const floatx4 dpn = dn * (1.f - nn * nn);
        const floatx4 dpr = dpn * pa * r * (1.f - r);
        const floatx4 dpz = dz * z * (1.f - z);
        carry = dh * z;
        dxk[0] = dpr; dxk[1] = dpz; dxk[2] = dpn;
        publish4(rsE, eoff, dpr);
        publish4(rsE, eoff + 4 * H, dpz);
        publish4(rsE, eoff + 8 * H, dpn * r);
        bsx[0] += dpr; bsx[1] += dpz; bsx[2] += dpn;
        bsh[0] += dpr; bsh[1] += dpz; bsh[2] += dpn * r;
      } else {
        floatx4 der;
#pragma unroll
        for (int i = 0; i < 4; i++) der[i] = MODE == kRelu ? (pap[i] > 0.f ? 1.f : 0.f) : (1.f - pap[i] * pap[i]);
        const floatx4 dp = dh * der;
        publish4(rsE, eoff, dp);
        bsx[0] += dp;
      }
    }
    if (p.sync == kSyncFlag) signal_flag(myflag, epoch);
    REC_TRACE(ks, 4);
    if (MODE == kGru && has_item) {
#pragma unroll
      for (int q = 0; q < NW; q++) st4(p.DX + grow + q * H, dxk[q]);
    }
    if (k > 0) prefetch(k - 1);
    __syncthreads();
    REC_TRACE(ks, 5);
  }
  // bias partial sums: reduce over n in a fixed order through LDS
  float *bs = red;  // reuse: [2][N][U][NW] floats
  if (has_item) {
#pragma unroll
    for (int q = 0; q < NW; q++)
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const long base = ((long)in_ * U + 4 * iq + i) * NW + q;
        bs[base] = bsx[q][i];
        bs[(long)N * U * NW + base] = (MODE == kGru) ? bsh[q][i] : bsx[q][i];
      }
  }
  __syncthreads();
  for (int q = tid; q < 2 * NW * U; q += NT) {
    const int part = q / (NW * U), rem = q - part * NW * U, gt = rem / U, u = rem - gt * U;
    float s = 0.f;
    for (int n = 0; n < N; n++) s += bs[(long)part * N * U * NW + ((long)n * U + u) * NW + gt];
    p.bias[((long)d * 2 + part) * NW * H + gt * H + u0 + u] = s;
  }
  if (bad && tid == 0) atomicOr(p.err, 1u);
}


// ---------------------------------------------------------------------------
// v4: XCD-local recurrences
// ---------------------------------------------------------------------------
// Grid = 8 * nwg; block b works as (dir = b & 7, g = b >> 3) when b & 7 < dirs,
// the others exit at once.  Under the observed round-robin dispatch the nwg
// (<= 32) workgroups of one direction then share one XCD and its L2, so the
// per-step all-gather of h (or dGates) is served by that L2 instead of the
// fabric.  This is checked, never assumed: every workgroup publishes its
// HW_REG_XCC_ID through the placement-independent form, and only when ALL
// workgroups of a direction read one id does that direction hand off through
// its L2 (plain payload and flag stores, which stay in the shared L2; sc1
// loads, which bypass the reading CU's L1).  Otherwise it uses the
// placement-independent form throughout (sc1 write-through payload and flag
// stores after every storing wave's vmcnt(0) and a barrier, sc1 loads:
// MI355X_MICROARCH.md "Valid forms", row 1).  Either way a step is
//   wait for the direction's nwg epoch flags (one sc1 poll per lane, wave 0)
//   -> sc1 16-B loads of the previous step straight into MFMA A registers
//   -> v_mfma_f32_16x16x4_f32 over the LDS-resident R slice (K split over
//      the 4 waves, reduced through LDS)
//   -> pointwise cell math, one (n, unit) element per thread
//   -> payload stores -> vmcnt(0) -> barrier -> lane 0 epoch flag.
// Epoch 1 is the placement probe; step k publishes epoch k + 2.

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xfu;
}

__device__ __forceinline__ float fsigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float ftanh(float x) { return 2.f * fsigm(2.f * x) - 1.f; }

__device__ __forceinline__ void put(float *q, float v, int local) {
  if (local) {
    __hip_atomic_store(reinterpret_cast<unsigned *>(q), __float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
  } else {
    __hip_atomic_store(reinterpret_cast<unsigned *>(q), __float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ __forceinline__ void signal_epoch(unsigned *flag, unsigned epoch, int local) {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0) {
    if (local) __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Placement probe: returns 1 iff every workgroup of direction d is on this XCD.
__device__ int probe_local(const RecParams &p, int d, int g, unsigned *myflag, int &bad, int *bad_lds,
                           int *loc_lds) {
  unsigned *xt = p.flags + 512 + d * p.nwg;
  const unsigned me = xcc_id() + 1u;
  if (threadIdx.x == 0) __hip_atomic_store(xt + g, me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  signal_epoch(myflag, 1u, 0);
  wait_flags(p.flags + d * p.nwg, p.nwg, 1u, p.err, bad, bad_lds);
  if (threadIdx.x < 64) {
    bool ok = true;
    for (int i = threadIdx.x; i < p.nwg; i += 64)
      ok &= __hip_atomic_load(xt + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == me;
    const bool all = __all(ok);
    if (threadIdx.x == 0) *loc_lds = (all && p.allow_local) ? 1 : 0;
  }
  __syncthreads();
  return *loc_lds;
}

constexpr int kMaxEPT = 4;  // (n, unit) elements per thread: N * U <= 1024

// Exchange image of one step, fragment-major: [dirs][KG][Npad][16] floats
// (KG = 16-wide k-groups).  One MFMA A fragment (16 rows x 16 k) is 1 KB of
// contiguous memory, so every hand-off load instruction moves whole 128-B
// lines; producers write 16 consecutive units of a row as 64 contiguous bytes.
// The row-major copies the rest of the layer needs (y, E) are written with
// plain stores off the critical path.
__device__ __forceinline__ long xoff(int d, int kg, int n, int j, int KG, int Npad) {
  return (((long)d * KG + kg) * Npad + n) * 16 + j;
}

// Hand-off loads + MFMA body of one step with compile-time trip counts: all
// loads first, then the MFMAs consume them in issue order, so the in-order
// vmcnt lets the first k-groups compute while the rest are in flight.
// Forward: acc[RT][CT] += h_{t-1}[rows][k] * R_slice^T[k][cols], K split over
// the 4 waves (wave w: k-groups w, w+4, ...).
template <int RT, int CT, int KGW>
__device__ __forceinline__ void fwd_step_mfma(floatx4 (&acc)[RT][kMaxCT], __amdgpu_buffer_rsrc_t rs, long dbase,
                                              int Npad, const float *Rs, int LDR, int w, int fr, int fq) {
  u32x4 af[KGW][RT];
#pragma unroll
  for (int i = 0; i < KGW; i++)
#pragma unroll
    for (int rt = 0; rt < RT; rt++)
      af[i][rt] = ld_sc1(rs, (unsigned)((dbase + ((long)(w + 4 * i) * Npad + rt * 16 + fr) * 16 + fq * 4) * 4));
#pragma unroll
  for (int i = 0; i < KGW; i++) {
    const int kg = w + 4 * i;
    floatx4 b[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ct++) b[ct] = ld4(Rs + (ct * 16 + fr) * LDR + kg * 16 + fq * 4);
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
      for (int ct = 0; ct < CT; ct++)
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
          acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[i][rt][s]), b[ct][s], acc[rt][ct],
                                                             0, 0, 0);
  }
}

// Backward: acc[RT] = dG_{t+1}[rows][kk] * R^T_slice[kk][units] over all nW*H
// kk (wave w: k-groups w, w+4, ...); NA accumulator sets interleaved so no
// MFMA waits on its predecessor, summed in a fixed order.
template <int RT, int KGW>
__device__ __forceinline__ void bwd_step_mfma(floatx4 (&acc)[RT], __amdgpu_buffer_rsrc_t rs, long dbase, int Npad,
                                              const float *RT_s, int LDK, int w, int fr, int fq) {
  constexpr int NA = (KGW % 4 == 0) ? 4 : (KGW % 2 == 0 ? 2 : 1);
  u32x4 af[KGW][RT];
#pragma unroll
  for (int i = 0; i < KGW; i++)
#pragma unroll
    for (int rt = 0; rt < RT; rt++)
      af[i][rt] = ld_sc1(rs, (unsigned)((dbase + ((long)(w + 4 * i) * Npad + rt * 16 + fr) * 16 + fq * 4) * 4));
  floatx4 part[NA][RT];
#pragma unroll
  for (int a = 0; a < NA; a++)
#pragma unroll
    for (int rt = 0; rt < RT; rt++) part[a][rt] = floatx4{0.f, 0.f, 0.f, 0.f};
  const float *brow = RT_s + fr * LDK + fq * 4;
#pragma unroll
  for (int i0 = 0; i0 < KGW; i0 += NA) {
    floatx4 b[NA];
#pragma unroll
    for (int a = 0; a < NA; a++) b[a] = ld4(brow + (w + 4 * (i0 + a)) * 16);
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
      for (int a = 0; a < NA; a++)
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
          part[a][rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[i0 + a][rt][s]), b[a][s],
                                                             part[a][rt], 0, 0, 0);
  }
#pragma unroll
  for (int rt = 0; rt < RT; rt++) {
    floatx4 t = part[0][rt];
#pragma unroll
    for (int a = 1; a < NA; a++) t += part[a][rt];
    acc[rt] = t;
  }
}

// generic (runtime trip count) versions of the same bodies
template <int RT>
__device__ __forceinline__ void fwd_step_generic(floatx4 (&acc)[RT][kMaxCT], __amdgpu_buffer_rsrc_t rs, long dbase,
                                                 int Npad, int KG, int CT, const float *Rs, int LDR, int w, int fr,
                                                 int fq) {
  for (int kg = w; kg < KG; kg += 4) {
    u32x4 af[RT];
#pragma unroll
    for (int rt = 0; rt < RT; rt++)
      af[rt] = ld_sc1(rs, (unsigned)((dbase + ((long)kg * Npad + rt * 16 + fr) * 16 + fq * 4) * 4));
#pragma unroll
    for (int ct = 0; ct < kMaxCT; ct++) {
      if (ct < CT) {
        const floatx4 b = ld4(Rs + (ct * 16 + fr) * LDR + kg * 16 + fq * 4);
#pragma unroll
        for (int s = 0; s < 4; s++)
#pragma unroll
          for (int rt = 0; rt < RT; rt++)
            acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[rt][s]), b[s], acc[rt][ct], 0, 0, 0);
      }
    }
  }
}
template <int RT>
__device__ __forceinline__ void bwd_step_generic(floatx4 (&acc)[RT], __amdgpu_buffer_rsrc_t rs, long dbase, int Npad,
                                                 int KG, const float *RT_s, int LDK, int w, int fr, int fq) {
  for (int kg = w; kg < KG; kg += 4) {
    u32x4 af[RT];
#pragma unroll
    for (int rt = 0; rt < RT; rt++)
      af[rt] = ld_sc1(rs, (unsigned)((dbase + ((long)kg * Npad + rt * 16 + fr) * 16 + fq * 4) * 4));
    const floatx4 b = ld4(RT_s + fr * LDK + kg * 16 + fq * 4);
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
      for (int rt = 0; rt < RT; rt++)
        acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(af[rt][s]), b[s], acc[rt], 0, 0, 0);
  }
}

// Everything else a step reads from or writes to HBM (next step's input
// projection / dy / saved activations, the row-major y / E copies) is issued
// right AFTER the step's hand-off loads have been consumed, never in front of
// them: a wave's vector memory operations complete in issue order.
template <int MODE, int RT>
__global__ __launch_bounds__(NT, 1) void rnn_fwd_rec4(RecParams p) {
  REC_TRACE_INIT;
  constexpr int NW = MODE == kLstm ? 4 : MODE == kGru ? 3 : 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int bad_lds, loc_lds;
  const int slot = blockIdx.x & 7, d = slot / p.xpd, g = (blockIdx.x >> 3) * p.xpd + slot % p.xpd;
  if (d >= p.dirs || g >= p.nwg) return;
  const int H = p.H, U = p.U, N = p.N, T = p.T, ncol = p.ncol, Npad = p.Npad;
  const int LDR = H + 4;
  const int u0 = g * U;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int CT = ncol / 16;
  const long ldy = (long)p.dirs * H, ldg = (long)p.dirs * NW * H;
  const int KG = H / 16;
  const long xstep = (long)p.dirs * KG * Npad * 16;  // floats of one step's exchange image
  float *Rs = smem;                      // [ncol][LDR]
  float *red = Rs + (long)ncol * LDR;    // [4][Npad][ncol]
  const float *Wd = p.w + d * p.pl_stride;
  const float *R = Wd + p.r_off;
  if (tid == 0) bad_lds = 0;
  for (int idx = tid; idx < ncol * H; idx += NT) {
    const int c = idx / H, k = idx - c * H;
    float v = 0.f;
    if (c < NW * U) {
      const int gt = c / U, u = c - gt * U;
      v = R[(long)(gt * H + u0 + u) * H + k];
    }
    Rs[c * LDR + k] = v;
  }
  const int items = N * U;
  float cst[kMaxEPT], hpv[kMaxEPT], gin[kMaxEPT][NW], gnx[kMaxEPT][NW], bR[kMaxEPT][NW];
  float act[kMaxEPT][NW], cnew[kMaxEPT], hval[kMaxEPT];
  auto gin_load = [&](int t, float (&dst)[kMaxEPT][NW]) {
#pragma unroll
    for (int j = 0; j < kMaxEPT; j++) {
      const int e = tid + j * NT, n = e / U, u = e - n * U;
      if (e < items) {
#pragma unroll
        for (int q = 0; q < NW; q++) dst[j][q] = p.G[((long)t * N + n) * ldg + (long)d * NW * H + q * H + u0 + u];
      }
    }
  };
  // row-major outputs of step t: y, and for the backward pass G (activations,
  // overwritten in place) and aux
  auto out_store = [&](int t) {
#pragma unroll
    for (int j = 0; j < kMaxEPT; j++) {
      const int e = tid + j * NT, n = e / U, u = e - n * U;
      if (e < items) {
        p.y[((long)t * N + n) * ldy + (long)d * H + u0 + u] = hval[j];
        if (MODE == kLstm || MODE == kGru) {
          const long grow = ((long)t * N + n) * ldg + (long)d * NW * H + u0 + u;
#pragma unroll
          for (int q = 0; q < NW; q++) p.G[grow + q * H] = act[j][q];
          p.aux[((long)t * N + n) * ldy + (long)d * H + u0 + u] = cnew[j];
        }
      }
    }
  };
#pragma unroll
  for (int j = 0; j < kMaxEPT; j++) {
    cst[j] = hpv[j] = cnew[j] = hval[j] = 0.f;
    const int e = tid + j * NT, u = e % U;
#pragma unroll
    for (int q = 0; q < NW; q++) {
      bR[j][q] = (MODE == kGru && e < items) ? Wd[p.bR_off + q * H + u0 + u] : 0.f;
      gin[j][q] = gnx[j][q] = act[j][q] = 0.f;
    }
  }
  gin_load(d == 0 ? 0 : T - 1, gin);
  int bad = 0;
  unsigned *myflag = p.flags + d * p.nwg + g;
  const int local = probe_local(p, d, g, myflag, bad, &bad_lds, &loc_lds);
  const int KGW = KG / 4;
  const int fast = (KG % 4 == 0 && KGW * RT <= 32 && (KGW == 8 || KGW == 4)) ? CT * 100 + KGW / 2 : 0;
  const long dbase = (long)d * KG * Npad * 16;
  int t_prev = -1;
  for (int k = 0; k < T && !bad; k++) {
    const int t = d == 0 ? k : T - 1 - k, tp = d == 0 ? t - 1 : t + 1;
    floatx4 acc[RT][kMaxCT];
#pragma unroll
    for (int a = 0; a < RT; a++)
#pragma unroll
      for (int b = 0; b < kMaxCT; b++) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    REC_TRACE(k, 0);
    if (k > 0) {
      wait_flags(p.flags + d * p.nwg, p.nwg, (unsigned)(k + 1), p.err, bad, &bad_lds);
      REC_TRACE(k, 1);
      const auto rs = rsrc(p.xch + (long)tp * xstep, (unsigned)(xstep * 4));
      switch (fast) {
        case 104: fwd_step_mfma<RT, 1, 8>(acc, rs, dbase, Npad, Rs, LDR, w, fr, fq); break;
        case 204: fwd_step_mfma<RT, 2, 8>(acc, rs, dbase, Npad, Rs, LDR, w, fr, fq); break;
        case 304: fwd_step_mfma<RT, 3, 8>(acc, rs, dbase, Npad, Rs, LDR, w, fr, fq); break;
        case 404: fwd_step_mfma<RT, 4, 8>(acc, rs, dbase, Npad, Rs, LDR, w, fr, fq); break;
        case 102: fwd_step_mfma<RT, 1, 4>(acc, rs, dbase, Npad, Rs, LDR, w, fr, fq); break;
        case 202: fwd_step_mfma<RT, 2, 4>(acc, rs, dbase, Npad, Rs, LDR, w, fr, fq); break;
        case 302: fwd_step_mfma<RT, 3, 4>(acc, rs, dbase, Npad, Rs, LDR, w, fr, fq); break;
        case 402: fwd_step_mfma<RT, 4, 4>(acc, rs, dbase, Npad, Rs, LDR, w, fr, fq); break;
        default: fwd_step_generic<RT>(acc, rs, dbase, Npad, KG, CT, Rs, LDR, w, fr, fq); break;
      }
    }
    asm volatile("" ::: "memory");
    // behind the hand-off loads: last step's row-major outputs, next step's
    // input projection
    if (t_prev >= 0) out_store(t_prev);
    if (k + 1 < T) gin_load(d == 0 ? t + 1 : t - 1, gnx);
#pragma unroll
    for (int rt = 0; rt < RT; rt++)
#pragma unroll
      for (int ct = 0; ct < kMaxCT; ct++)
        if (ct < CT)
#pragma unroll
          for (int r = 0; r < 4; r++)
            red[((long)w * Npad + rt * 16 + fq * 4 + r) * ncol + ct * 16 + fr] = acc[rt][ct][r];
    if (p.trace) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      REC_TRACE_W(k, 10);
    }
    __syncthreads();
    REC_TRACE(k, 3);
    float *xt = p.xch + (long)t * xstep;
#pragma unroll
    for (int j = 0; j < kMaxEPT; j++) {
      const int e = tid + j * NT;
      if (e >= items) continue;
      const int n = e / U, u = e - n * U;
      float rh[NW];
#pragma unroll
      for (int q = 0; q < NW; q++) {
        const int c = q * U + u;
        rh[q] = ((red[((long)0 * Npad + n) * ncol + c] + red[((long)1 * Npad + n) * ncol + c]) +
                 red[((long)2 * Npad + n) * ncol + c]) + red[((long)3 * Npad + n) * ncol + c];
      }
      float h;
      if (MODE == kLstm) {
        act[j][0] = fsigm(gin[j][0] + rh[0]);
        act[j][1] = fsigm(gin[j][1] + rh[1]);
        act[j][2] = ftanh(gin[j][2] + rh[2]);
        act[j][3] = fsigm(gin[j][3] + rh[3]);
        cst[j] = act[j][1] * cst[j] + act[j][0] * act[j][2];
        cnew[j] = cst[j];
        h = act[j][3] * ftanh(cst[j]);
      } else if (MODE == kGru) {
        act[j][0] = fsigm(gin[j][0] + rh[0] + bR[j][0]);
        act[j][1] = fsigm(gin[j][1] + rh[1] + bR[j][1]);
        cnew[j] = rh[2] + bR[j][2];
        act[j][2] = ftanh(gin[j][2] + act[j][0] * cnew[j]);
        h = (1.f - act[j][1]) * act[j][2] + act[j][1] * hpv[j];
        hpv[j] = h;
      } else {
        const float pre = gin[j][0] + rh[0];
        h = MODE == kRelu ? fmaxf(pre, 0.f) : ftanh(pre);
      }
      hval[j] = h;
      const int uu = u0 + u;
      put(xt + xoff(d, uu >> 4, n, uu & 15, KG, Npad), h, local);
    }
    signal_epoch(myflag, (unsigned)(k + 2), local);
    REC_TRACE(k, 4);
#pragma unroll
    for (int j = 0; j < kMaxEPT; j++)
#pragma unroll
      for (int q = 0; q < NW; q++) gin[j][q] = gnx[j][q];
    t_prev = t;
    __syncthreads();  // red[] is rewritten by the next step
    REC_TRACE(k, 5);
  }
  if (t_prev >= 0 && !bad) out_store(t_prev);
  if (bad && tid == 0) atomicOr(p.err, 1u);
}

template <int MODE, int RT>
__global__ __launch_bounds__(NT, 1) void rnn_bwd_rec4(RecParams p) {
  REC_TRACE_INIT;
  constexpr int NW = MODE == kLstm ? 4 : MODE == kGru ? 3 : 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int bad_lds, loc_lds;
  const int slot = blockIdx.x & 7, d = slot / p.xpd, g = (blockIdx.x >> 3) * p.xpd + slot % p.xpd;
  if (d >= p.dirs || g >= p.nwg) return;
  const int H = p.H, U = p.U, N = p.N, T = p.T, Npad = p.Npad;
  const int K = NW * H, LDK = K + 4;
  const int KG = K / 16;
  const long xstep = (long)p.dirs * KG * Npad * 16;
  const int u0 = g * U;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const long ldy = (long)p.dirs * H, ldg = (long)p.dirs * NW * H;
  float *RT_s = smem;                       // [16][LDK]: RT_s[u][kk] = R[kk][u0+u], rows >= U zero
  float *red = RT_s + (long)16 * LDK;       // [4][Npad][16]
  const float *Wd = p.w + d * p.pl_stride;
  const float *R = Wd + p.r_off;
  if (tid == 0) bad_lds = 0;
  for (int idx = tid; idx < 16 * K; idx += NT) {
    const int kk = idx / 16, u = idx - kk * 16;
    RT_s[u * LDK + kk] = u < U ? R[(long)kk * H + u0 + u] : 0.f;
  }
  const int items = N * U;
  // per element: current step's operands (c*), the next step's (n*), and the
  // row-major dGates of the previous step waiting to be stored (e*, dxk)
  float carry[kMaxEPT], bsx[kMaxEPT][NW], bsh[kMaxEPT][NW], dxk[kMaxEPT][NW], eg[kMaxEPT][NW];
  float cg[kMaxEPT][NW], cdy[kMaxEPT], ca[kMaxEPT], cap[kMaxEPT];
  float ng[kMaxEPT][NW], ndy[kMaxEPT], na[kMaxEPT], nap[kMaxEPT];
#pragma unroll
  for (int j = 0; j < kMaxEPT; j++) {
    carry[j] = cdy[j] = ca[j] = cap[j] = ndy[j] = na[j] = nap[j] = 0.f;
#pragma unroll
    for (int q = 0; q < NW; q++) bsx[j][q] = bsh[j][q] = cg[j][q] = ng[j][q] = dxk[j][q] = eg[j][q] = 0.f;
  }
  auto prefetch = [&](int k) {  // operands of forward-order step k into n*
    const int t = d == 0 ? k : T - 1 - k, tp = d == 0 ? t - 1 : t + 1;
#pragma unroll
    for (int j = 0; j < kMaxEPT; j++) {
      const int e = tid + j * NT;
      if (e >= items) continue;
      const int n = e / U, u = e - n * U;
      const long yrow = ((long)t * N + n) * ldy + (long)d * H + u0 + u;
      const long grow = ((long)t * N + n) * ldg + (long)d * NW * H + u0 + u;
      const long prow = ((long)tp * N + n) * ldy + (long)d * H + u0 + u;
      ndy[j] = p.dy[yrow];
      if (MODE == kLstm || MODE == kGru) {
#pragma unroll
        for (int q = 0; q < NW; q++) ng[j][q] = p.G[grow + q * H];
        na[j] = p.aux[yrow];
      }
      if (MODE == kLstm) nap[j] = k > 0 ? p.aux[prow] : 0.f;
      else if (MODE == kGru) nap[j] = k > 0 ? p.y[prow] : 0.f;
      else nap[j] = p.y[yrow];
    }
  };
  auto rotate = [&]() {
#pragma unroll
    for (int j = 0; j < kMaxEPT; j++) {
      cdy[j] = ndy[j]; ca[j] = na[j]; cap[j] = nap[j];
#pragma unroll
      for (int q = 0; q < NW; q++) cg[j][q] = ng[j][q];
    }
  };
  auto e_store = [&](int t) {  // row-major dGates of step t (E; GRU also DX)
#pragma unroll
    for (int j = 0; j < kMaxEPT; j++) {
      const int e = tid + j * NT;
      if (e >= items) continue;
      const int n = e / U, u = e - n * U;
      const long grow = ((long)t * N + n) * ldg + (long)d * NW * H + u0 + u;
#pragma unroll
      for (int q = 0; q < NW; q++) p.E[grow + q * H] = eg[j][q];
      if (MODE == kGru) {
#pragma unroll
        for (int q = 0; q < NW; q++) p.DX[grow + q * H] = dxk[j][q];
      }
    }
  };
  prefetch(T - 1);
  rotate();
  int bad = 0;
  unsigned *myflag = p.flags + d * p.nwg + g;
  const int local = probe_local(p, d, g, myflag, bad, &bad_lds, &loc_lds);
  const int KGW = KG / 4;
  const int fast = (KG % 4 == 0 && KGW * RT <= 32 &&
                    (KGW == 32 || KGW == 24 || KGW == 16 || KGW == 12 || KGW == 8 || KGW == 4)) ? KGW : 0;
  const long dbase = (long)d * KG * Npad * 16;
  int t_prev = -1;
  for (int k = T - 1; k >= 0 && !bad; k--) {
    const int t = d == 0 ? k : T - 1 - k;
    const int tn = d == 0 ? t + 1 : t - 1;
    const int ks = T - 1 - k;             // steps done before this one
    floatx4 acc[RT];
#pragma unroll
    for (int a = 0; a < RT; a++) acc[a] = floatx4{0.f, 0.f, 0.f, 0.f};
    REC_TRACE(ks, 0);
    if (ks > 0) {
      wait_flags(p.flags + d * p.nwg, p.nwg, (unsigned)(ks + 1), p.err, bad, &bad_lds);
      REC_TRACE(ks, 1);
      const auto rs = rsrc(p.xch + (long)tn * xstep, (unsigned)(xstep * 4));
      switch (fast) {
        case 32: bwd_step_mfma<RT, 32>(acc, rs, dbase, Npad, RT_s, LDK, w, fr, fq); break;
        case 24: bwd_step_mfma<RT, 24>(acc, rs, dbase, Npad, RT_s, LDK, w, fr, fq); break;
        case 16: bwd_step_mfma<RT, 16>(acc, rs, dbase, Npad, RT_s, LDK, w, fr, fq); break;
        case 12: bwd_step_mfma<RT, 12>(acc, rs, dbase, Npad, RT_s, LDK, w, fr, fq); break;
        case 8: bwd_step_mfma<RT, 8>(acc, rs, dbase, Npad, RT_s, LDK, w, fr, fq); break;
        case 4: bwd_step_mfma<RT, 4>(acc, rs, dbase, Npad, RT_s, LDK, w, fr, fq); break;
        default: bwd_step_generic<RT>(acc, rs, dbase, Npad, KG, RT_s, LDK, w, fr, fq); break;
      }
    }
    asm volatile("" ::: "memory");
    // behind the hand-off loads: next step's operands, last step's row-major dGates
    if (k > 0) prefetch(k - 1);
    if (t_prev >= 0) e_store(t_prev);
#pragma unroll
    for (int rt = 0; rt < RT; rt++)
#pragma unroll
      for (int r = 0; r < 4; r++) red[((long)w * Npad + rt * 16 + fq * 4 + r) * 16 + fr] = acc[rt][r];
    if (p.trace) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      REC_TRACE_W(ks, 10);
    }
    __syncthreads();
    REC_TRACE(ks, 3);
    float *xt = p.xch + (long)t * xstep;
#pragma unroll
    for (int j = 0; j < kMaxEPT; j++) {
      const int e = tid + j * NT;
      if (e >= items) continue;
      const int n = e / U, u = e - n * U;
      const float dhr = ((red[((long)0 * Npad + n) * 16 + u] + red[((long)1 * Npad + n) * 16 + u]) +
                         red[((long)2 * Npad + n) * 16 + u]) + red[((long)3 * Npad + n) * 16 + u];
      float dh = cdy[j] + dhr;
      const int uu = u0 + u;
      if (MODE == kLstm) {
        const float ig = cg[j][0], fg = cg[j][1], gg = cg[j][2], og = cg[j][3];
        const float tc = ftanh(ca[j]);
        const float dO = dh * tc;
        const float dc = dh * og * (1.f - tc * tc) + carry[j];
        eg[j][0] = dc * gg * ig * (1.f - ig);
        eg[j][1] = dc * cap[j] * fg * (1.f - fg);
        eg[j][2] = dc * ig * (1.f - gg * gg);
        eg[j][3] = dO * og * (1.f - og);
        carry[j] = dc * fg;
      } else if (MODE == kGru) {
        dh += carry[j];
        const float r = cg[j][0], z = cg[j][1], nn = cg[j][2];
        const float dn = dh * (1.f - z), dz = dh * (cap[j] - nn);
        const float dpn = dn * (1.f - nn * nn);
        const float dpr = dpn * ca[j] * r * (1.f - r);
        const float dpz = dz * z * (1.f - z);
        carry[j] = dh * z;
        dxk[j][0] = dpr; dxk[j][1] = dpz; dxk[j][2] = dpn;
        eg[j][0] = dpr; eg[j][1] = dpz; eg[j][2] = dpn * r;
        bsh[j][0] += dpr; bsh[j][1] += dpz; bsh[j][2] += dpn * r;
      } else {
        const float der = MODE == kRelu ? (cap[j] > 0.f ? 1.f : 0.f) : (1.f - cap[j] * cap[j]);
        eg[j][0] = dh * der;
      }
#pragma unroll
      for (int q = 0; q < NW; q++) {
        const int kk = q * H + uu;
        put(xt + xoff(d, kk >> 4, n, kk & 15, KG, Npad), eg[j][q], local);
        bsx[j][q] += (MODE == kGru) ? dxk[j][q] : eg[j][q];
      }
    }
    signal_epoch(myflag, (unsigned)(ks + 2), local);
    REC_TRACE(ks, 4);
    rotate();
    t_prev = t;
    __syncthreads();
    REC_TRACE(ks, 5);
  }
  if (t_prev >= 0 && !bad) e_store(t_prev);
  // bias partial sums: reduce over n in a fixed order through LDS
  float *bs = red;  // reuse: [2][N][U][NW] floats (fits: see lds sizing)
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kMaxEPT; j++) {
    const int e = tid + j * NT;
    if (e >= items) continue;
    const int n = e / U, u = e - n * U;
#pragma unroll
    for (int q = 0; q < NW; q++) {
      const long base = ((long)n * U + u) * NW + q;
      bs[base] = bsx[j][q];
      bs[(long)N * U * NW + base] = (MODE == kGru) ? bsh[j][q] : bsx[j][q];
    }
  }
  __syncthreads();
  for (int q = tid; q < 2 * NW * U; q += NT) {
    const int part = q / (NW * U), rem = q - part * NW * U, gt = rem / U, u = rem - gt * U;
    float s = 0.f;
    for (int n = 0; n < N; n++) s += bs[(long)part * N * U * NW + ((long)n * U + u) * NW + gt];
    p.bias[((long)d * 2 + part) * NW * H + gt * H + u0 + u] = s;
  }
  if (bad && tid == 0) atomicOr(p.err, 1u);
}

// ---------------------------------------------------------------------------
// v6 backward: reduce-scatter hand-off, split-fp16 MFMA
// ---------------------------------------------------------------------------
// WG (dir, g) owns units u0..u0+U-1 and the K = nW*U rows of R that feed those
// units' gates.  Per step it
//   (1) sums the partial dh of its units from every producer WG of its
//       direction (published the step before; fixed summation order),
//   (2) does the pointwise cell backward of its (n, unit) elements (one per
//       thread) -> dGates [N x K],
//   (3) multiplies dGates [16 x K] by its R rows [K x H] on the matrix cores,
//       every wave owning H/4 output columns (no cross-wave reduction), and
//   (4) publishes that partial dh of ALL H units, fp32, in the MFMA C-fragment
//       layout [producer][col tile][lane][4] (1 KB per 16 x 16 tile).
// Per WG and step 32 KB are read and 32 KB written (BLSTM-512, N=16) instead of
// the 128 KB dGates all-gather of v4.
//
// Split-fp16 products ("fp16x3"): both operands are scaled by powers of two
// (R slice: one exponent per WG, from its max |R|; dGates: one exponent per
// row, from the row's max over the WG's K columns) so the largest magnitude
// lands in [2^13, 2^14), and split as x = hi + lo with hi = fp16(x),
// lo = fp16(x - hi).  acc += hi_a hi_b + hi_a lo_b + lo_a hi_b on
// v_mfma_f32_16x16x32_f16 (products exact, fp32 accumulation), then the exact
// power-of-two unscale.  Each operand keeps 22 significant bits relative to
// its row / slice maximum; the dropped lo*lo term is 2^-22 of it -- the same
// order as fp32 rounding of the accumulated terms.  5.3x fewer MFMA cycles
// than v_mfma_f32_16x16x4_f32 for the same product.
//
// R lives in registers for the whole launch (the B fragments of the wave's
// H/64 column tiles, hi and lo); dGates goes through a 4.5 KB LDS image.
// Hand-off as v4 (sc1 payload stores, vmcnt(0), barrier, sc1 epoch flag;
// sc1 loads) into a per-step image that is never rewritten within a launch.
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
// products of the v6 recurrences: split-fp16 (fp32-class) or bf16
enum { kPrecX3 = 0, kPrecBf16 = 1, kPrecX3S = 2 };
// kPrecX3S: split-fp16 with the hi and lo parts stacked in ONE 16-row MFMA
// operand -- for row groups of <= 8 sequences, whose tiles leave rows 8..15
// empty: A = [hi rows 0..7; lo rows 0..7], acc += A B_hi + A B_lo, then row r
// + row r + 8 = hi B_hi + hi B_lo + lo B_hi + lo B_lo (all four terms: 2 MFMAs
// per block instead of 3, and the lo x lo term the 3-MFMA form drops)

// rows r + 8 of a 16 x 16 C fragment (lanes 32..63) added into rows r (lanes
// 0..31); lanes 32..63 are left with garbage
__device__ __forceinline__ float fold_rows8(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return x + __uint_as_float(r[1]);
}
// max over each aligned group of U (8, 16, 32) lanes, all lanes active
__device__ __forceinline__ float group_maxU(float v, int U) {
  v = U > 8 ? group_max16(v) : group_max8(v);
  if (U > 16) v = fmaxf(v, __shfl_xor(v, 16));
  return v;
}


// v6 flag words: one 128-B line per (direction, workgroup), so that the
// producers' flag stores and the consumers' polls spread over L2 / memory
// channels instead of hammering one line.
constexpr int kFlagStride = 32;  // words
// word of the flag area where an XCD-pinned backward recurrence's workgroups
// OR in 1 << XCC_ID (words 1008 / 1009: weight-gradient tile counters)
constexpr int kXcdWord = 1016;
constexpr int kResWord = 1017;  // v6 recurrence: workgroups resident so far (beside_recurrence)
constexpr int kGateWord = 1018;  // blocks of its residency gate that left (rnn_resident_gate)
__device__ __forceinline__ unsigned *flag6(const RecParams &p, int grp, int d, int g, int nwg) {
  return p.flags + 1024 + (((long)grp * p.dirs + d) * nwg + g) * kFlagStride;
}
// aggregated epoch of (row group, direction) for the streamed GEMMs of an
// XCD-pinned recurrence: one line each, 256 lines past the flag lines
__device__ __forceinline__ unsigned *agg_flag6(const RecParams &p, int grp, int d) {
  return p.flags + 1024 + (256 + (long)grp * p.dirs + d) * kFlagStride;
}
__device__ __forceinline__ void wait_flags6(const unsigned *f0, int nwg, unsigned epoch, unsigned *err, int &bad,
                                            int *bad_lds, int sleep = 1) {
  if (threadIdx.x < 64) {
    int spins = 0;
    while (true) {
      bool ok = true;
      for (int i = threadIdx.x; i < nwg; i += 64)
        ok &= __hip_atomic_load(f0 + (long)i * kFlagStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= epoch;
      if (__all(ok)) break;
      if (++spins > kSpinLimit ||
          ((spins & 255) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        bad = 1;
        if (threadIdx.x == 0) {
          *bad_lds = 1;
          if (spins > kSpinLimit) atomicOr(err, 0x10000u);  // this wait ran out of time itself
        }
        break;
      }
      if (sleep) __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (*bad_lds) bad = 1;
}
// Per-wave wait (the forward's flagged hand-off): a wave waits only for the
// producers whose rows IT loads -- lane j polls producer prod (-1: none) --
// and goes on to its own loads and MFMAs while the other waves still wait, so
// the hand-off of the last producer to publish costs only the loads of the
// waves that read it.  No workgroup barrier (the step's next one follows the
// K reduction); a timeout sets *bad_lds for the barrier after.
__device__ __forceinline__ bool wave_wait_prod(const unsigned *f0, int prod, unsigned epoch, unsigned *err,
                                               int *bad_lds, int sleep) {
  int spins = 0;
  while (true) {
    const bool ok =
        prod < 0 || __hip_atomic_load(f0 + (long)prod * kFlagStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= epoch;
    if (__all(ok)) return true;
    if (++spins > kSpinLimit ||
        ((spins & 255) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
      if ((threadIdx.x & 63) == 0) *bad_lds = 1;
      return false;
    }
    if (sleep) __builtin_amdgcn_s_sleep(1);
  }
}

// Placement probe of a v6 launch in XCD-slot mapping: 1 iff every workgroup of
// direction d reads the same HW_REG_XCC_ID (then the hand-off may stay in that
// XCD's L2: plain payload and flag stores, sc1 loads).  Publishes epoch 1.
__device__ int probe6(const RecParams &p, int grp, int d, int g, int nwg, int &bad, int *bad_lds, int *loc_lds) {
  unsigned *ids = p.flags + 512 + (grp * p.dirs + d) * nwg;
  const unsigned me = xcc_id() + 1u;
  if (threadIdx.x == 0) __hip_atomic_store(ids + g, me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  signal_epoch(flag6(p, grp, d, g, nwg), 1u, 0);
  wait_flags6(flag6(p, grp, d, 0, nwg), nwg, 1u, p.err, bad, bad_lds);
  if (threadIdx.x < 64) {
    bool ok = true;
    for (int i = threadIdx.x; i < nwg; i += 64)
      ok &= __hip_atomic_load(ids + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == me;
    const bool all = __all(ok);
    if (threadIdx.x == 0) *loc_lds = all ? 1 : 0;
  }
  __syncthreads();
  return *loc_lds;
}

// 4-byte LDS-DMA (global_load_lds_dword): lane l's dword to LDS byte address
// lds + 4 l.  Inline asm, so that the compiler's wait-count pass does not see
// it: a pending LDS-DMA there merges into the other waves' code paths of
// the same kernel and turns their exact vmcnt waits into vmcnt(0).  The
// issuing wave waits for it with explicit s_waitcnt and reads none of it.
// M0 (a reserved register) is saved and restored inside the statement.
__device__ __forceinline__ void dma_lds_dword(const float *g, unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(lds)
      : "memory");
}

// the same, system-coherent (sc1): data written by another XCD while this
// kernel runs (a concurrent producer's write-through stores)
__device__ __forceinline__ void dma_lds_dword_sc1(const void *g, unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off sc1\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(lds)
      : "memory");
}

// A system-coherent 4-byte load that has landed when the statement ends, and
// a write-through 4-byte store, both invisible to the compiler's wait-count
// pass: memory operations it can see on the IO waves' paths merge into the
// hand-off waves' paths at the barriers and make their exact waits
// conservative (measured: a forward with such polls 2.06 -> 2.4 us/step).
__device__ __forceinline__ unsigned ld_u32_sc1_now(const unsigned *g) {
  unsigned v;
  asm volatile("global_load_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(g) : "memory");
  return v;
}
__device__ __forceinline__ void st_u32_sc1(unsigned *g, unsigned v) {
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(g), "v"(v) : "memory");
}

// Workgroup barrier for LDS hand-offs.  RAW = true: the LDS writes drained
// and s_barrier, without __syncthreads' fence -- with LDS-DMA in flight the
// fence waits for every outstanding vector memory operation (vmcnt(0)),
// which would turn the IO waves' G fetch three steps ahead into one step and
// hold the hand-off waves on their own stores.  Only for barriers that order
// LDS traffic alone.
template <bool RAW>
__device__ __forceinline__ void lds_barrier() {
  if constexpr (RAW) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  } else {
    __syncthreads();
  }
}

// exponent s with max * 2^s in [2^13, 2^14) (s = 14 for max == 0)
__device__ __forceinline__ int split_exp(float mx) {
  int e = 0;
  (void)frexpf(mx, &e);
  return 14 - e;
}

__device__ __forceinline__ void split16(float x, _Float16 &hi, _Float16 &lo) {
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}

// Generalisation (row groups, wide workgroups, bf16): the N sequences are
// split into RG = ceil(N / 16) groups of 16 rows, each an independent
// recurrence on its own dirs x NWG workgroups, flag lines and exchange images
// (block b -> direction b % dirs, workgroup (b / dirs) % NWG, group
// b / (dirs NWG)); a workgroup of NTH = 256 or 512 threads owns U = 8, 16 or
// 32 units (one (row, unit) element per thread, NTH / 64 waves each owning
// H / (16 NTH / 64) output column tiles).  P = kPrecBf16 multiplies bf16
// dGates by a bf16 R slice instead of the split-fp16 pair (one MFMA per
// block, no scaling; partial dh stay fp32).
#ifndef KCTC_PIPE_STK
#define KCTC_PIPE_STK 1
#endif
// stacked backward: partial-dh stores pipelined behind the next tile's MFMAs
constexpr bool kPipeStk = KCTC_PIPE_STK != 0;
#ifndef KCTC_EARLY_E
#define KCTC_EARLY_E 1
#endif
// bf16 backward: the previous step's dGates stores under the hand-off loads
constexpr bool kEarlyE = KCTC_EARLY_E != 0;
template <int MODE, int U, int H, int NTH, int P>
__global__ __launch_bounds__(NTH, 1) void rnn_bwd_rec6(RecParams p) {
  REC_TRACE_INIT;
  constexpr int NW = MODE == kLstm ? 4 : 3;
  constexpr int NWV = NTH / 64;
  constexpr int K = NW * U, KB = (K + 31) / 32, AP = KB * 32 + 8;  // A image row pitch (halves)
  constexpr int CTW = H / (16 * NWV), CTT = H / 16, NWG = H / U;
  static_assert(CTW * 16 * NWV == H, "output column tiles per wave");
  static_assert(16 * U <= NTH, "one (row, unit) element per thread");
  constexpr int POS = 4 * U;       // 16-B chunks of the own column tiles per producer
  constexpr int NGRP = NTH / POS;  // producer groups
  constexpr int PER = NWG / NGRP;  // producers summed per group
  static_assert(NWG % NGRP == 0, "producer groups");
  constexpr bool BF = P == kPrecBf16;
  constexpr bool STK = P == kPrecX3S;  // dGates hi / lo stacked in one 16-row A image (groups of <= 8 rows)
  // split-fp16: the cell's coefficients before the hand-off (see kc below);
  // bf16 (configs[4], every wave an element wave) measured faster with the
  // whole pointwise backward in the cell (3.65 vs 3.46 us/step)
  constexpr bool PRE = !BF;
  using AT = typename std::conditional<BF, __bf16, _Float16>::type;
  using AV = typename std::conditional<BF, bf16x8, halfx8>::type;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int bad_lds, loc_lds;
  __shared__ int rowexp[16];
  __shared__ float wmax[NWV];
  // xpd = 1: XCD-slot mapping (block b -> direction b & 7, so a direction's 32
  // workgroups share one XCD under round-robin dispatch; checked by probe6;
  // one row group only); else block b -> (group, workgroup, direction)
  const int dirs = p.dirs;
  const int d = p.xpd ? (blockIdx.x & 7) % dirs : blockIdx.x % dirs;
  const int g = p.xpd ? (blockIdx.x >> 3) : (blockIdx.x / dirs) % NWG;
  const int grp = p.xpd ? (blockIdx.x & 7) / dirs : blockIdx.x / (dirs * NWG);
  if (d >= dirs || g >= NWG || grp >= p.rg) return;
  // resident: counted for the exchange's residency gate (rnn_comm_gate) and
  // in the launch's own word for the side launches beside it (beside_recurrence)
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(p.flags + kResWord, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (p.reg) {
      __hip_atomic_fetch_add(reinterpret_cast<unsigned long long *>(p.reg + 4), 1ull, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      if (p.xpd) __hip_atomic_fetch_or(p.reg + 2, 1u << xcc_id(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // rnn_pinned_xcds
    }
  }
  // rows n0 .. nend-1 of the batch (p.gs <= 16 of the 16 MFMA rows)
  const int N = p.N, T = p.T, n0 = grp * p.gs, nend = min(N, n0 + p.gs);
  const int u0 = g * U, ct_own = u0 >> 4, fr0 = u0 & 15;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const long ldy = (long)dirs * H, ldg = (long)dirs * NW * H;
  // floats per producer block (16 x H) + 256 B, so that the 1-KB chunks a
  // consumer reads from consecutive producers fall in different L2 channels
  // bf16 mode (p.bfpart): the partials travel as bf16 (8 B per lane and tile,
  // summed in fp32 by the consumer), half the bytes of the fp32 images
  const bool bfp = BF && p.bfpart;
  const long PSTR = bfp ? (long)CTT * 64 * 2 + 64 : (long)CTT * 64 * 4 + 64;
  const int LW = bfp ? 2 : 4;  // floats-worth per lane and tile
  const long xgrp = (long)dirs * NWG * PSTR;  // one row group's images of a step
  const long xstep = xgrp * p.rg;
  AT *Ahi = reinterpret_cast<AT *>(smem);  // [16][AP]
  AT *Alo = Ahi + 16 * AP;                 // x3 only
  float *red = reinterpret_cast<float *>(Alo + (BF ? 0 : 16 * AP));  // [NGRP][POS][4]
  // streamed consumer: this step's dGates tile [16][NW * U] (DX for GRU), then
  // written through with 16-B stores after the step's signal
  float *estg = red + (NTH * 4 > 2 * 16 * U * NW ? NTH * 4 : 2 * 16 * U * NW);
  const float *Wd = p.w + d * p.pl_stride;
  const float *R = Wd + p.r_off;
  if (tid == 0) bad_lds = 0;
  for (int i = tid; i < (BF ? 16 : 32) * AP; i += NTH) Ahi[i] = (AT)0.f;  // the image(s), padding included
  // ---- R slice -> B fragments in registers (x3: scaled hi/lo; bf16: as is) ----
  // K order of the dGates operand: split-fp16 paths unit-major (k = u NW + q:
  // an element's NW gates are adjacent halves, one 8-B LDS write per part),
  // bf16 gate-major (k = q U + u)
  constexpr bool KUM = !BF;
  auto rval = [&](int kk, int col) -> float {
    if (kk >= K) return 0.f;
    const int q = KUM ? kk % NW : kk / U, u = KUM ? kk / NW : kk - (kk / U) * U;
    return R[(long)(q * H + u0 + u) * H + col];
  };
  int sB = 0;
  if constexpr (!BF) {
    float mx = 0.f;
#pragma unroll
    for (int c = 0; c < CTW; c++)
#pragma unroll
      for (int kb = 0; kb < KB; kb++)
#pragma unroll
        for (int j = 0; j < 8; j++) mx = fmaxf(mx, fabsf(rval(kb * 32 + fq * 8 + j, (w * CTW + c) * 16 + fr)));
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    if (lane == 0) wmax[w] = mx;
    __syncthreads();
    float m4 = wmax[0];
#pragma unroll
    for (int i = 1; i < NWV; i++) m4 = fmaxf(m4, wmax[i]);
    sB = split_exp(m4);
  }
  AV bhi[CTW][KB], blo[BF ? 1 : CTW][BF ? 1 : KB];
  if constexpr (!BF) {
#pragma unroll
    for (int c = 0; c < CTW; c++)
#pragma unroll
      for (int kb = 0; kb < KB; kb++)
#pragma unroll
        for (int j = 0; j < 8; j++) {
          _Float16 h, l;
          split16(ldexpf(rval(kb * 32 + fq * 8 + j, (w * CTW + c) * 16 + fr), sB), h, l);
          bhi[c][kb][j] = h;
          blo[c][kb][j] = l;
        }
  }
  // bf16: filled after the start-up wait (probe6) below -- filled here, hipcc
  // sank the conversions past that wait loop with all 8 x KB x CTW fp32
  // values live and spilled the 512-thread GRU kernel to scratch (before the
  // step loop, but a kernel with scratch must run alone: rec6_scratch_free)
  // ---- per-element state: thread tid <-> (row n0 + en, unit u0 + eu) ----
  const bool has_e = tid < 16 * U;
  const int en = tid / U, eu = tid - en * U;
  const int n = n0 + en;
  const bool live = has_e && n < nend;
  float carry = 0.f, bsx[NW], bsh[NW], dxk[NW], eg[NW], cg[NW], ng[NW], cmx[NW], cme[NW];
  float cdy = 0.f, ca = 0.f, cap = 0.f, ndy = 0.f, na = 0.f, nap = 0.f;
  // The cell's coefficients -- everything of the pointwise backward that does
  // not depend on the hand-off -- computed from the step's forward values
  // after the previous step's publish (while the other producers' epochs are
  // on their way), so that the cell after the hand-off is a few FMAs:
  //   LSTM: dc = dh kc[0] + carry, dG_q = dc kc[1+q] (q < 3), dG_3 = dh kc[4], carry = dc kc[5]
  //   GRU : dh += carry, dX_q = dh kc[q], dE_2 = dh kc[3], carry = dh kc[4]
  float kc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto coef = [&]() {
    if (MODE == kLstm) {
      const float ig = cg[0], fg = cg[1], gg = cg[2], og = cg[3];
      const float tc = ftanh(ca);
      kc[0] = og * (1.f - tc * tc);
      kc[1] = gg * ig * (1.f - ig);
      kc[2] = cap * fg * (1.f - fg);
      kc[3] = ig * (1.f - gg * gg);
      kc[4] = tc * og * (1.f - og);
      kc[5] = fg;
    } else {
      const float r = cg[0], z = cg[1], nn = cg[2];
      const float kn = (1.f - z) * (1.f - nn * nn);
      kc[0] = kn * ca * r * (1.f - r);
      kc[1] = (cap - nn) * z * (1.f - z);
      kc[2] = kn;
      kc[3] = kn * r;
      kc[4] = z;
    }
  };
  // bias and column-maximum bookkeeping of the step's dGates, and their LDS
  // stage for the next step's row writes
  auto book = [&]() {
#pragma unroll
    for (int q = 0; q < NW; q++) {
      bsx[q] += (MODE == kGru) ? dxk[q] : eg[q];
      if (MODE == kGru) bsh[q] += eg[q];
      if (live) {  // column maxima for the weight GEMMs' packed transposes
        cmx[q] = fmaxf(cmx[q], fabsf(MODE == kGru ? dxk[q] : eg[q]));
        if (MODE == kGru) cme[q] = fmaxf(cme[q], fabsf(eg[q]));
      }
    }
    if (p.e_sc1 || (BF && p.dxt != nullptr)) {
#pragma unroll
      for (int q = 0; q < NW; q++) estg[en * NW * U + q * U + eu] = MODE == kGru ? dxk[q] : eg[q];
      if (MODE == kGru && BF && p.dxt != nullptr) {
#pragma unroll
        for (int q = 0; q < NW; q++) estg[16 * NW * U + en * NW * U + q * U + eu] = eg[q];
      }
    }
  };
#pragma unroll
  for (int q = 0; q < NW; q++) bsx[q] = bsh[q] = dxk[q] = eg[q] = cg[q] = ng[q] = cmx[q] = cme[q] = 0.f;
  // this element's operand columns as per-lane pointers, opaque to the
  // compiler: they stay in VGPRs and the kernel-argument bases die here
  // (the loop's scalar registers spill otherwise)
  const float *dy_e = p.dy + (long)n * ldy + (long)d * H + u0 + eu;
  const float *g_e = p.G + (long)n * ldg + (long)d * NW * H + u0 + eu;
  const float *aux_e = p.aux + (long)n * ldy + (long)d * H + u0 + eu;
  const float *prv_e = (MODE == kLstm ? p.aux : p.y) + (long)n * ldy + (long)d * H + u0 + eu;
  asm volatile("" : "+v"(dy_e), "+v"(g_e), "+v"(aux_e), "+v"(prv_e));
  auto prefetch = [&](int k) {  // operands of forward-order step k into n*
    if (!live) return;
    const int t = d == 0 ? k : T - 1 - k, tp = d == 0 ? t - 1 : t + 1;
    const long yo = (long)t * N * ldy, go = (long)t * N * ldg, po = (long)tp * N * ldy;
    ndy = dy_e[yo];
#pragma unroll
    for (int q = 0; q < NW; q++) ng[q] = g_e[go + q * H];
    na = aux_e[yo];
    nap = k > 0 ? prv_e[po] : 0.f;
  };
  auto rotate = [&]() {
    cdy = ndy; ca = na; cap = nap;
#pragma unroll
    for (int q = 0; q < NW; q++) cg[q] = ng[q];
  };
  // bf16 packed operands (p.dxt): the step's DX tile is staged in estg and the
  // GRU's E tile in estg2 during the cell phase; the next step writes them as
  // 16-B bf16 chunks (DX rows; DX^T and E^T columns of 8 frames)
  float *estg2 = estg + 16 * NW * U;
  const bool pk = BF && p.dxt != nullptr;
  auto pk_store = [&](int tt) {
    if constexpr (BF) {
      constexpr int RCH = NW * U / 8;  // 16-B row chunks per row
      const long TNl = (long)T * N, G4 = (long)NW * H;
      const long f0 = (long)tt * N + n0;
      // DX rows: thread -> (row, chunk)
      for (int i = tid; i < 16 * RCH; i += NTH) {
        const int rn = i / RCH, ch = i - rn * RCH, q = (ch * 8) / U, u = (ch * 8) % U;
        if (n0 + rn >= nend) continue;
        bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = (__bf16)estg[rn * NW * U + q * U + u + j];
        *reinterpret_cast<bf16x8 *>(p.dxr + ((long)d * TNl + f0 + rn) * G4 + q * H + u0 + u) = v;
      }
      // DX^T (and E^T) columns: thread -> (column, 8-frame half); aligned 16-B
      // chunks when the 8 frames are whole, else per frame.  E^T shifted
      // (eshift): frames of step 0 (direction 0) / T - 1 (direction 1) drop out
      const bool vec8 = (N % 8 == 0) && (n0 % 8 == 0);
      const int narr = (MODE == kGru || p.eshift) ? 2 : 1;
      const long esh = p.eshift ? (d == 0 ? -(long)N : (long)N) : 0;
      const bool edrop = p.eshift && (d == 0 ? tt == 0 : tt == T - 1);
      for (int i = tid; i < narr * NW * U * 2; i += NTH) {
        const int which = i / (NW * U * 2), rem = i - which * NW * U * 2, col = rem >> 1, half = rem & 1;
        if (which && edrop) continue;
        const float *src = (which && MODE == kGru) ? estg2 : estg;
        __bf16 *dst = (which ? p.et : p.dxt) + ((long)d * G4 + (col / U) * H + u0 + col % U) * p.kbt64 + f0 + half * 8 +
                      (which ? esh : 0);
        const int r0 = half * 8;
        if (vec8 && n0 + r0 + 8 <= nend) {
          bf16x8 v;
#pragma unroll
          for (int j = 0; j < 8; j++) v[j] = (__bf16)src[(r0 + j) * NW * U + col];
          *reinterpret_cast<bf16x8 *>(dst) = v;
        } else {
          for (int j = 0; j < 8; j++)
            if (n0 + r0 + j < nend) dst[j] = (__bf16)src[(r0 + j) * NW * U + col];
        }
      }
    }
  };
  auto e_store = [&](int t) {  // row-major dGates of step t (E; GRU also DX)
    if (pk) {
      pk_store(t);
      return;
    }
    if (!live) return;
    const long grow = ((long)t * N + n) * ldg + (long)d * NW * H + u0 + eu;
    if (p.e_sc1) {  // DX (== E for LSTM) went out through estg already
      if (MODE == kGru) {
#pragma unroll
        for (int q = 0; q < NW; q++) p.E[grow + q * H] = eg[q];
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < NW; q++) p.E[grow + q * H] = eg[q];
    if (MODE == kGru) {
#pragma unroll
      for (int q = 0; q < NW; q++) p.DX[grow + q * H] = dxk[q];
    }
  };
  // consumer chunk of this thread: position pos (of the own column tiles'
  // C-fragment chunks) of producers pg, pg + NGRP, ...
  const int pos = tid % POS, pg = tid / POS;
  const int pln = U >= 16 ? pos : (pos >> 3) * 16 + fr0 + (pos & 7);
  const long coff = (long)grp * xgrp + (long)d * NWG * PSTR + ((long)ct_own * 64 + pln) * LW + (long)pg * PSTR;
  // a C-fragment lane holds rows 4 (lane / 16) .. +3 of the group: quads past N
  // are neither stored nor loaded (a group of fewer than 16 sequences moves
  // only its own rows).  STK (transposed, U = 16): chunk j = 8 (unit / 4) +
  // row of a tile holds units 4 (j / 8) .. +3 of row j % 8, chunks 32..63 unused
  const bool crow_live = STK ? (pln < 32 && n0 + (pln & 7) < nend) : n0 + 4 * ((pln & 63) >> 4) < nend;
  const bool prow_live = STK ? (fr < 8 && n0 + fr < nend) : n0 + 4 * fq < nend;
  // where element (en, eu) finds its sum: own tile eu / 16, lane (en / 4) * 16
  // + (eu % 16) (U = 8: compacted to 8 per row quad), register en % 4
  const int epos = STK ? (eu >> 2) * 8 + en : (eu >> 4) * 64 + (en >> 2) * (U < 16 ? U : 16) + (eu & 15);
  const int ereg = STK ? (eu & 3) : (en & 3);
  prefetch(T - 1);
  rotate();
  if constexpr (PRE) coef();
  int bad = 0;
  unsigned *myflag = flag6(p, grp, d, g, NWG);
  // XCD-slot launches keep the hand-off in the XCD's L2 (plain flag stores
  // other XCDs do not see).  For the streamed dx GEMM running on the other
  // XCDs, workgroup 0 of each (row group, direction) publishes ONE aggregated
  // sc1 epoch (agg_flag6): after the first barrier of step ks it has seen every
  // producer's epoch ks + 1, whose signals drained their rows of step ks - 2,
  // so it stores ks + 1 ("rows of step k complete at epoch k + 3").  One line
  // per direction instead of 32 for up to ~100 polling GEMM blocks.
  unsigned *gflag = (p.xpd && p.e_sc1 && g == 0) ? agg_flag6(p, grp, d) : nullptr;
  // and where it runs, for the streamed GEMM's blocks (on_pinned_xcd)
  // (before any wait on another workgroup: a residency gate block on this XCD
  // leaves on it, rnn_resident_gate)
  if (p.xpd && tid == 0) atomicOr(p.flags + kXcdWord, 1u << xcc_id());
  if (tid == 0) loc_lds = 0;
  const int local = (p.xpd && p.allow_local) ? probe6(p, grp, d, g, NWG, bad, &bad_lds, &loc_lds) : 0;
  if constexpr (BF) {
    auto fill = [&]() {
#pragma unroll
      for (int c = 0; c < CTW; c++)
#pragma unroll
        for (int kb = 0; kb < KB; kb++)
#pragma unroll
          for (int j = 0; j < 8; j++) bhi[c][kb][j] = (__bf16)rval(kb * 32 + fq * 8 + j, (w * CTW + c) * 16 + fr);
    };
    fill();
  }
  if (trc_ && tid == 0) trc_[9] = (unsigned long long)(local + 1);  // step 0, slot 9
  // Self-tagged hand-off (fp32 partials, XCD-local slot, ring of two step
  // images set to tag 1 before the launch): the producer's partial-dh words
  // carry ((step >> 1) & 1) in their LSB, the consumers re-load a chunk until
  // all its words carry the step's tag.  No per-step drain, signal barrier,
  // flag store or flag poll -- the poll IS the payload load.  Ring safety as
  // before: a producer writes slot ks % 2 only after it has read every
  // consumer's step ks - 1 words, stored after that consumer's loads of step
  // ks - 2 had returned.
  const bool dtag = !BF && p.dtag && local && p.ring == 2;
  // step t's DX rows for a streaming consumer on other XCDs, from the LDS
  // stage: written through (sc1) as whole 16-B chunks, 4 lanes per
  // contiguous 64-B run (4-B write-through stores per element cost ~8 us per
  // step); the next signal drains them, so they are complete at epoch t + 3
  auto e_sc1_store = [&](int tt) {
    constexpr int CPR = NW * U / 4;  // chunks per row
    // self-tagged (issued after the first barrier): the LAST 16 CPR threads,
    // i.e. the waves past the element waves when there are any, store while
    // the element waves do the cell
    const int et = dtag ? tid - (NTH - 16 * CPR) : tid;
    const int rn = et >= 0 ? et / CPR : 16, c = et - rn * CPR;
    if (rn < 16 && n0 + rn < nend) {
      const int q = (c * 4) / U, u = (c * 4) % U;
      const u32x4 v = *reinterpret_cast<const u32x4 *>(estg + rn * NW * U + c * 4);
      const int off = (int)(((long)(n0 + rn) * ldg + (long)d * NW * H + q * H + u0 + u) * 4);
      __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(p.DX + (long)tt * N * ldg, (unsigned)(N * ldg * 4)), off, 0, 16);
    }
  };
  int t_prev = -1;
  for (int k = T - 1; k >= 0 && !bad; k--) {
    const int t = d == 0 ? k : T - 1 - k;
    const int ks = T - 1 - k;  // steps done before this one
    REC_TRACE(ks, 0);
    if (ks > 0) {
      if (dtag) {
        // self-tagged: no flags; the poll below is the wait
      } else {
        wait_flags6(flag6(p, grp, d, 0, NWG), NWG, (unsigned)(ks + 1), p.err, bad, &bad_lds, p.poll_sleep);
      }
      REC_TRACE(ks, 1);
      REC_TRACE_W(ks, 16);
      const auto rs = rsrc(p.xch + (long)(p.ring ? (ks - 1) & 1 : ks - 1) * xstep, (unsigned)(xstep * 4));  // (ring: 2 images)
      floatx4 sm = floatx4{0.f, 0.f, 0.f, 0.f};
      if (bfp) {
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        u32x2 v[PER];
        // unconditional (a dead row quad past the buffer: zeros), so that the
        // work below overlaps them
#pragma unroll
        for (int i = 0; i < PER; i++)
          v[i] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(
                     rs, crow_live ? (int)((coff + (long)i * NGRP * PSTR) * 4) : 0x7fff0000, 0, 16 /* sc1 */));
        if constexpr (PRE) {
          __builtin_amdgcn_sched_barrier(0);
          coef();  // while the hand-off loads are in flight
          __builtin_amdgcn_sched_barrier(0);
        } else if (kEarlyE) {
          // bf16: the previous step's dGates rows / packed operands (its
          // cell's estg stage, complete since the MFMA phase's barrier) while
          // the hand-off loads are in flight, instead of after them
          __builtin_amdgcn_sched_barrier(0);
          e_store(t_prev);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int i = 0; i < PER; i++) {
          const bf16x4 b = __builtin_bit_cast(bf16x4, v[i]);
#pragma unroll
          for (int j = 0; j < 4; j++) sm[j] += (float)b[j];
        }
      } else {
        u32x4 v[PER];
        // unconditional loads (a dead row quad at an offset past the buffer:
        // the hardware returns zeros), so that the compiler counts them
        // exactly and the coefficients below overlap them
        auto hoff = [&](int i) { return crow_live ? (unsigned)((coff + (long)i * NGRP * PSTR) * 4) : 0x7fff0000u; };
#pragma unroll
        for (int i = 0; i < PER; i++) v[i] = ld_sc1(rs, hoff(i));
        if constexpr (PRE) {
          __builtin_amdgcn_sched_barrier(0);
          coef();  // while the hand-off loads are in flight
          // (pinned here: IR passes had sunk the coefficients past the loads' wait)
#pragma unroll
          for (int q = 0; q < 6; q++) asm volatile("" : "+v"(kc[q]));
          __builtin_amdgcn_sched_barrier(0);
        }
        if (dtag) {
          // every word of step ks - 1 carries tag ((ks - 1) >> 1) & 1 in its
          // LSB; a chunk still holding step ks - 3's words (the other tag) is
          // loaded again.  4-B words are single-copy atomic, so a 16-B load
          // that tears between the two steps is caught word by word.
          const unsigned want = (unsigned)((ks - 1) >> 1) & 1u;
          auto ready = [&]() {
            unsigned bad4 = 0u;
#pragma unroll
            for (int i = 0; i < PER; i++) bad4 |= (v[i][0] ^ want) | (v[i][1] ^ want) | (v[i][2] ^ want) | (v[i][3] ^ want);
            return !crow_live || (bad4 & 1u) == 0u;
          };
          int spins = 0;
          while (!__all(ready())) {  // (not all there yet: the wave loads all its chunks again)
            if (++spins > kSpinLimit ||
                ((spins & 255) == 0 &&
                 __builtin_amdgcn_readfirstlane(__hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)))) {
              bad = 1;
              if (lane == 0) bad_lds = 1;
              break;
            }
            if (p.poll_sleep) __builtin_amdgcn_s_sleep(1);
            asm volatile("" ::: "memory");
#pragma unroll
            for (int i = 0; i < PER; i++) v[i] = ld_sc1(rs, hoff(i));
          }
        }
        sm = __builtin_bit_cast(floatx4, v[0]);
#pragma unroll
        for (int i = 1; i < PER; i++) sm += __builtin_bit_cast(floatx4, v[i]);
      }
      st4(red + (long)(pg * POS + pos) * 4, sm);
      REC_TRACE(ks, 2);
      REC_TRACE_W(ks, 24);
      // behind this step's hand-off loads: the write-through copies for the
      // streamed dx GEMM -- the previous step's dGates rows (staged in LDS)
      // and the epoch the last signal drained (step ks - 2's rows).  Issued
      // after the signal instead, they were still in flight at the next flag
      // poll, which waits for every older store (one vmcnt for loads and stores)
      // (self-tagged: after the barrier below, which orders it behind the
      // previous step's book() writes of estg -- no signal barrier in between)
      if (p.e_sc1 && !dtag) e_sc1_store(t_prev);
    }
    asm volatile("" ::: "memory");
    // behind the hand-off loads: next step's operands, last step's row-major dGates
    if (t_prev >= 0 && !(kEarlyE && !PRE && bfp && ks > 0)) e_store(t_prev);
    if (k > 0) prefetch(k - 1);
    __syncthreads();
    REC_TRACE(ks, 8);
    if (bad_lds) bad = 1;
    // self-tagged: every producer's words of step ks - 1 were stored after its
    // poll of step ks - 2 had retired (in-order vmcnt) its write-through rows
    // of step ks - 3 -> epoch ks (rows of step k out at epoch k + 3);
    // flagged: its signal of step ks - 1 drained the rows of step ks - 2
    if (gflag && ks > 0 && tid == 0)
      __hip_atomic_store(gflag, (unsigned)(dtag ? ks : ks + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (dtag && p.e_sc1 && ks > 0) e_sc1_store(t_prev);
    if (has_e) {
      float dhr = 0.f;
      if (ks > 0) {
        // all NGRP reads in flight before the first add (one LDS latency,
        // not NGRP), then the fixed-order sum
        float rr[NGRP];
#pragma unroll
        for (int gg = 0; gg < NGRP; gg++) rr[gg] = red[(long)(gg * POS + epos) * 4 + ereg];
        __builtin_amdgcn_sched_group_barrier(0x100, NGRP, 0);
#pragma unroll
        for (int gg = 0; gg < NGRP; gg++) dhr += rr[gg];
      }
      float dh = cdy + dhr;
      if constexpr (PRE) {
        if (MODE == kLstm) {
          const float dc = dh * kc[0] + carry;
          eg[0] = dc * kc[1];
          eg[1] = dc * kc[2];
          eg[2] = dc * kc[3];
          eg[3] = dh * kc[4];
          carry = dc * kc[5];
        } else {
          dh += carry;
          dxk[0] = dh * kc[0]; dxk[1] = dh * kc[1]; dxk[2] = dh * kc[2];
          eg[0] = dxk[0]; eg[1] = dxk[1]; eg[2] = dh * kc[3];
          carry = dh * kc[4];
        }
      } else if (MODE == kLstm) {
        const float ig = cg[0], fg = cg[1], gg = cg[2], og = cg[3];
        const float tc = ftanh(ca);
        const float dO = dh * tc;
        const float dc = dh * og * (1.f - tc * tc) + carry;
        eg[0] = dc * gg * ig * (1.f - ig);
        eg[1] = dc * cap * fg * (1.f - fg);
        eg[2] = dc * ig * (1.f - gg * gg);
        eg[3] = dO * og * (1.f - og);
        carry = dc * fg;
      } else {
        dh += carry;
        const float r = cg[0], z = cg[1], nn = cg[2];
        const float dn = dh * (1.f - z), dz = dh * (cap - nn);
        const float dpn = dn * (1.f - nn * nn);
        const float dpr = dpn * ca * r * (1.f - r);
        const float dpz = dz * z * (1.f - z);
        carry = dh * z;
        dxk[0] = dpr; dxk[1] = dpz; dxk[2] = dpn;
        eg[0] = dpr; eg[1] = dpz; eg[2] = dpn * r;
      }
      float m = 0.f;
#pragma unroll
      for (int q = 0; q < NW; q++) m = fmaxf(m, fabsf(eg[q]));
      if constexpr (!PRE) book();
      if constexpr (BF) {
#pragma unroll
        for (int q = 0; q < NW; q++) Ahi[en * AP + q * U + eu] = (__bf16)eg[q];
      } else {
        const int se = split_exp(group_maxU(m, U));
        // unit-major K: the element's NW gates are halves eu NW .. eu NW + NW - 1
        // of its row (STK: hi in row en < 8, lo in row en + 8)
        _Float16 hh[4], hl[4];
#pragma unroll
        for (int q = 0; q < 4; q++) hh[q] = hl[q] = (_Float16)0.f;
#pragma unroll
        for (int q = 0; q < NW; q++) split16(ldexpf(eg[q], se), hh[q], hl[q]);
        _Float16 *dhi = Ahi + en * AP + eu * NW;
        _Float16 *dlo = STK ? Ahi + (en + 8) * AP + eu * NW : Alo + en * AP + eu * NW;
        if (!STK || en < 8) {
          if constexpr (NW == 4) {
            typedef _Float16 half4 __attribute__((ext_vector_type(4)));
            *reinterpret_cast<half4 *>(dhi) = half4{hh[0], hh[1], hh[2], hh[3]};
            *reinterpret_cast<half4 *>(dlo) = half4{hl[0], hl[1], hl[2], hl[3]};
          } else {
#pragma unroll
            for (int q = 0; q < NW; q++) {
              dhi[q] = hh[q];
              dlo[q] = hl[q];
            }
          }
        }
        if (eu == 0) rowexp[en] = se + sB;
      }
    }
    REC_TRACE(ks, 12);
    __syncthreads();
    REC_TRACE(ks, 3);
    if (STK && k > 0 && kPipeStk) {
      // partial dh of all units for the next step, stacked hi / lo: tile c's
      // four MFMAs, then -- while tile c + 1's run -- its fold, scaling, tag
      // and 16-B store, as one straight-line block per cache policy (the
      // store of a dead lane goes past the buffer's end and is dropped)
      const auto ro = rsrc(p.xch + (long)(p.ring ? ks & 1 : ks) * xstep, (unsigned)(xstep * 4));
      const long obase = (long)grp * xgrp + (long)(d * NWG + g) * PSTR;
      const unsigned tg = (unsigned)(ks >> 1) & 1u;
      const int e1 = -rowexp[fr & 7];
      AV ah[KB];
#pragma unroll
      for (int kb = 0; kb < KB; kb++) ah[kb] = *reinterpret_cast<const AV *>(Ahi + fr * AP + kb * 32 + fq * 8);
      auto phase = [&](auto aux_c) {
        constexpr int aux = decltype(aux_c)::value;
        floatx4 acc[CTW];
#pragma unroll
        for (int c = 0; c < CTW; c++) {
          acc[c] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kb = 0; kb < KB; kb++) {  // the order of the interleaved version: hi, lo per k block
            acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bhi[c][kb], ah[kb], acc[c], 0, 0, 0);
            acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(blo[c][kb], ah[kb], acc[c], 0, 0, 0);
          }
        }
#pragma unroll
        for (int c = 0; c < CTW; c++) {
          floatx4 o;
#pragma unroll
          for (int i = 0; i < 4; i++) {
            float v = acc[c][i] + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc[c][i]), 0x128, 0xF, 0xF, true));
            v = ldexpf(v, e1);
            o[i] = __uint_as_float((__float_as_uint(v) & ~1u) | tg);
          }
          const int slot = fq * 8 + (fr & 7);
          const int off = prow_live ? (int)((obase + ((long)(w * CTW + c) * 64 + slot) * LW) * 4) : 0x7ffffff0;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), ro, off, 0, aux);
        }
        // pipeline: MFMAs of tiles 0 and 1, then per tile c the fold + store
        // of tile c - 1 ... interleaved with tile c + 1's MFMAs
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * KB, 0);  // tile 0 (2 KB MFMAs a tile)
#pragma unroll
        for (int c = 1; c < CTW; c++) {
          __builtin_amdgcn_sched_group_barrier(0x008, KB, 0);  // tile c (first half)
          __builtin_amdgcn_sched_group_barrier(0x002, 12, 0);  // tile c - 1: fold, scale, tag
          __builtin_amdgcn_sched_group_barrier(0x008, KB, 0);  // tile c (second half)
          __builtin_amdgcn_sched_group_barrier(0x040, 1, 0);   // tile c - 1: store
        }
        __builtin_amdgcn_sched_group_barrier(0x002, 12, 0);  // last tile
        __builtin_amdgcn_sched_group_barrier(0x040, 1, 0);
      };
      if (local) phase(std::integral_constant<int, 0>{});
      else phase(std::integral_constant<int, 16>{});
    } else if (BF && k > 0 && kPipeStk && bfp) {
      // bf16 with bf16 partials (configs[4]): the same pipeline -- tile c's KB
      // MFMAs, then its bf16 pack and 8-B store behind tile c + 1's
      const auto ro = rsrc(p.xch + (long)(p.ring ? ks & 1 : ks) * xstep, (unsigned)(xstep * 4));
      const long obase = (long)grp * xgrp + (long)(d * NWG + g) * PSTR;
      AV ah[KB];
#pragma unroll
      for (int kb = 0; kb < KB; kb++) ah[kb] = *reinterpret_cast<const AV *>(Ahi + fr * AP + kb * 32 + fq * 8);
      auto phase = [&](auto aux_c) {
        constexpr int aux = decltype(aux_c)::value;
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        floatx4 acc[CTW];
#pragma unroll
        for (int c = 0; c < CTW; c++) {
          acc[c] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kb = 0; kb < KB; kb++) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[kb], bhi[c][kb], acc[c], 0, 0, 0);
        }
#pragma unroll
        for (int c = 0; c < CTW; c++) {
          bf16x4 b;
#pragma unroll
          for (int i = 0; i < 4; i++) b[i] = (__bf16)acc[c][i];
          const int off = prow_live ? (int)((obase + ((long)(w * CTW + c) * 64 + lane) * LW) * 4) : 0x7ffffff0;
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, b), ro, off, 0, aux);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, KB, 0);  // tile 0
#pragma unroll
        for (int c = 1; c < CTW; c++) {
          __builtin_amdgcn_sched_group_barrier(0x008, KB, 0);  // tile c
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);   // tile c - 1: bf16 pack
          __builtin_amdgcn_sched_group_barrier(0x040, 1, 0);   // tile c - 1: store
        }
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // last tile
        __builtin_amdgcn_sched_group_barrier(0x040, 1, 0);
      };
      if (local) phase(std::integral_constant<int, 0>{});
      else phase(std::integral_constant<int, 16>{});
    } else if (k > 0) {  // partial dh of all units for the next step
      floatx4 acc[CTW];
#pragma unroll
      for (int c = 0; c < CTW; c++) acc[c] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < KB; kb++) {
        const AV ah = *reinterpret_cast<const AV *>(Ahi + fr * AP + kb * 32 + fq * 8);
        if constexpr (BF) {
#pragma unroll
          for (int c = 0; c < CTW; c++) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bhi[c][kb], acc[c], 0, 0, 0);
        } else if constexpr (STK) {
          // transposed: C^T[unit][row'] = R_slice^T dG^T, row' < 8 hi, >= 8 lo
          // (the R fragments as the A operand: same registers, A[unit][k])
#pragma unroll
          for (int c = 0; c < CTW; c++) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bhi[c][kb], ah, acc[c], 0, 0, 0);
#pragma unroll
          for (int c = 0; c < CTW; c++) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(blo[c][kb], ah, acc[c], 0, 0, 0);
        } else {
          const AV al = *reinterpret_cast<const AV *>(Alo + fr * AP + kb * 32 + fq * 8);
#pragma unroll
          for (int c = 0; c < CTW; c++) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bhi[c][kb], acc[c], 0, 0, 0);
#pragma unroll
          for (int c = 0; c < CTW; c++) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, blo[c][kb], acc[c], 0, 0, 0);
#pragma unroll
          for (int c = 0; c < CTW; c++) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bhi[c][kb], acc[c], 0, 0, 0);
        }
      }
      if constexpr (STK) {  // columns 8..15 (lo rows) onto 0..7: one DPP add (row_ror:8) per register
#pragma unroll
        for (int c = 0; c < CTW; c++)
#pragma unroll
          for (int i = 0; i < 4; i++)  // (mov_dpp with bound_ctrl: combined into one v_add_f32_dpp)
            acc[c][i] += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc[c][i]), 0x128, 0xF, 0xF, true));
      }
      int ex[4] = {0, 0, 0, 0};
      if constexpr (STK) {
        const int e1 = -rowexp[fr & 7];  // one row per lane
#pragma unroll
        for (int i = 0; i < 4; i++) ex[i] = e1;
      } else if constexpr (!BF) {
#pragma unroll
        for (int i = 0; i < 4; i++) ex[i] = -rowexp[fq * 4 + i];
      }
      // a ring of >= 2 images is safe: every workgroup is a consumer of every
      // producer, so before a producer writes slot ks % ring at step ks it saw
      // all flags of step ks - 1, i.e. every consumer had finished reading
      // that slot's previous contents (step ks - ring, read during ks - ring + 1)
      const auto ro = rsrc(p.xch + (long)(p.ring ? ks & 1 : ks) * xstep, (unsigned)(xstep * 4));
      const long obase = (long)grp * xgrp + (long)(d * NWG + g) * PSTR;
      // fp32 partials carry the step tag ((ks >> 1) & 1) in their LSB in every
      // mode (the self-tagged hand-off reads it; the others keep the same
      // arithmetic, so that pinned and unpinned runs stay bit-identical)
      const unsigned tg = (unsigned)(ks >> 1) & 1u;
#pragma unroll
      for (int c = 0; c < CTW; c++) {
        floatx4 o;
#pragma unroll
        for (int i = 0; i < 4; i++) {
          o[i] = BF ? acc[c][i] : ldexpf(acc[c][i], ex[i]);
          if (!bfp) o[i] = __uint_as_float((__float_as_uint(o[i]) & ~1u) | tg);
        }
        const int slot = STK ? (fq * 8 + (fr & 7)) : lane;  // STK: compact chunks of the 8 live columns
        const int off = (int)((obase + ((long)(w * CTW + c) * 64 + slot) * LW) * 4);
        // local: plain stores keep the lines in the XCD's shared L2, where the
        // consumers' sc1 loads find them; else write-through (sc1)
        if (!prow_live) {
        } else if (bfp) {
          typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
          bf16x4 b;
#pragma unroll
          for (int i = 0; i < 4; i++) b[i] = (__bf16)o[i];
          if (local) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, b), ro, off, 0, 0);
          else __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, b), ro, off, 0, 16);
        } else if (local) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), ro, off, 0, 0);
        } else {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), ro, off, 0, 16);
        }
      }
    }
    // off the hand-off path (behind the partial-dh stores, during their
    // drain): bias and column-maximum bookkeeping, the dGates stage for the
    // next step's row writes (read after the publish barrier)
    if constexpr (PRE) {
      __builtin_amdgcn_sched_barrier(0);
      if (has_e) book();
    }
    REC_TRACE(ks, 7);
    if (!dtag) signal_epoch(myflag, (unsigned)(ks + 2), local);
    REC_TRACE(ks, 4);
    rotate();
    t_prev = t;
    REC_TRACE(ks, 5);
  }
  if (dtag) __syncthreads();  // the last step's book() writes of estg, before e_sc1_store reads them
  if (t_prev >= 0 && !bad) e_store(t_prev);
  if (!bad) {
    if (p.e_sc1 && t_prev >= 0) e_sc1_store(t_prev);
    signal_epoch(myflag, (unsigned)(T + 2), 0);  // the last step's rows are out
    if (gflag) {  // every producer's last rows are out
      wait_flags6(flag6(p, grp, d, 0, NWG), NWG, (unsigned)(T + 2), p.err, bad, &bad_lds, p.poll_sleep);
      if (!bad && tid == 0) __hip_atomic_store(gflag, (unsigned)(T + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // bias partial sums of this row group: reduce over its rows in a fixed
  // order through LDS; the host adds the groups in order
  float *bs = red;  // [2][16][U][NW] floats
  __syncthreads();
  if (has_e) {
#pragma unroll
    for (int q = 0; q < NW; q++) {
      const long b0 = ((long)en * U + eu) * NW + q;
      bs[b0] = live ? bsx[q] : 0.f;
      bs[(long)16 * U * NW + b0] = live ? ((MODE == kGru) ? bsh[q] : bsx[q]) : 0.f;
    }
  }
  __syncthreads();
  for (int q = tid; q < 2 * NW * U; q += NTH) {
    const int part = q / (NW * U), rem = q - part * NW * U, gt = rem / U, u = rem - gt * U;
    float s2 = 0.f;
    for (int r = 0; r < 16; r++) s2 += bs[(long)part * 16 * U * NW + ((long)r * U + u) * NW + gt];
    p.bias[(((long)grp * dirs + d) * 2 + part) * NW * H + gt * H + u0 + u] = s2;
  }
  if (p.cmax) {  // column maxima over all frames (this group's rows, through LDS; max over groups)
    constexpr int NP = MODE == kGru ? 2 : 1;
    __syncthreads();
    if (has_e) {
#pragma unroll
      for (int q = 0; q < NW; q++) {
        bs[((long)en * U + eu) * NW + q] = cmx[q];
        if (MODE == kGru) bs[(long)16 * U * NW + ((long)en * U + eu) * NW + q] = cme[q];
      }
    }
    __syncthreads();
    for (int q = tid; q < NP * NW * U; q += NTH) {
      const int part = q / (NW * U), rem = q - part * NW * U, gt = rem / U, u = rem - gt * U;
      float m2 = 0.f;
      for (int r = 0; r < 16; r++) m2 = fmaxf(m2, bs[(long)part * 16 * U * NW + ((long)r * U + u) * NW + gt]);
      unsigned *dst = p.cmax + (long)part * dirs * NW * H + (long)d * NW * H + gt * H + u0 + u;
      if (p.rg > 1) atomicMax(dst, __float_as_uint(m2));  // non-negative floats order as their bits
      else *dst = __float_as_uint(m2);
    }
  }
  if (bad && tid == 0) atomicOr(p.err, 1u);
}

// ---------------------------------------------------------------------------
// v6 forward: split-fp16 MFMA over an fp16 hi/lo all-gather of h
// ---------------------------------------------------------------------------
// WG (dir, g) owns units u0..u0+U-1; per step it multiplies h_{t-1} [16 x H]
// by its R slice (the nW*U gate rows of its units) on
// v_mfma_f32_16x16x32_f16 with the split-fp16 products of the v6 backward
// (R scaled per WG, h scaled by 2^14: |h| <= 1 for LSTM / GRU), K split over
// the 4 waves and reduced through LDS in a fixed order, then does the cell
// update of its (n, unit) elements and publishes h_t as the fp16 hi/lo pair
// of its units.  The exchange image of a step is A-fragment-major:
// [dir][kb = k/32][hi|lo][16 rows][32 k] halves (1 KB per fragment), the same
// 64 KB per step as the fp32 image of v4; a consumer lane loads 16 B of hi
// and 16 B of lo per 32-k block.  The R slice lives in registers (B
// fragments) for the whole launch.  Hand-off as v4 (sc1 stores, vmcnt(0),
// barrier, sc1 epoch flag; sc1 loads).
// Generalised like rnn_bwd_rec6: row groups of 16 sequences (block b ->
// direction b % dirs, workgroup (b / dirs) % NWG, group b / (dirs NWG); each
// group has its own flag lines and step images), NTH = 256 or 512 threads (K
// split over NTH / 64 waves), U up to 32; P = kPrecBf16 exchanges h as bf16
// and multiplies by a bf16 R slice (one MFMA per block, no scaling).
template <int MODE, int U, int H, int NTH, int P>
__global__ __launch_bounds__(NTH, 1) void rnn_fwd_rec6(RecParams p) {
  REC_TRACE_INIT;
  constexpr int NW = MODE == kLstm ? 4 : 3;
  constexpr int NWV = NTH / 64;
  // P & 4: IO waves.  The upper half of the waves neither waits for the
  // hand-off nor multiplies: they load the input projection rows (G) of the
  // coming steps and pass them through LDS.  A wave's vmcnt counts its loads
  // and stores in order, so a G load (HBM latency) issued by a hand-off wave
  // held up that wave's next flag poll / hand-off loads / publish drain
  // (measured: forward 2.38 -> 1.89 us/step with the G loads left out)
  constexpr bool IOW = (P & 4) != 0;
  // the row-major outputs through the IO waves too: measured slower (forward
  // 2.46 -> 2.52 us/step; the IO waves' waits then delay the post-cell barrier)
  constexpr bool IO_OUT = false;
  constexpr int PR = P & 3;
  constexpr int CW = IOW ? NWV / 2 : NWV;  // hand-off (compute) waves
  constexpr int NC = NW * U, CT = (NC + 15) / 16, RP = CT * 16 + 1;  // red row pitch (floats)
  constexpr int KB = H / 32, KBW = (KB + CW - 1) / CW, NWG = H / U;
  constexpr int CH = U / 8;  // 16-B chunks of a published row part
  constexpr bool BF = PR == kPrecBf16;
  constexpr bool STK = PR == kPrecX3S;  // hi / lo stacked in one 16-row A operand (groups of <= 8 rows)
  constexpr int NP = BF ? 1 : 2;  // parts of an exchanged h: hi (+ lo)
  static_assert(16 * U <= NTH, "one (row, unit) element per thread");
  static_assert(!IOW || (16 * U == CW * 64 && NW <= 4 && NP * 16 * U / 8 <= 64),
                "IO waves: the elements fill the compute waves, one publishing wave");
  using AT = typename std::conditional<BF, __bf16, _Float16>::type;
  using AV = typename std::conditional<BF, bf16x8, halfx8>::type;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int bad_lds, loc_lds;
  __shared__ float wmax[NWV];
  const int dirs = p.dirs;
  // xpd = 1: XCD-slot mapping as rnn_bwd_rec6 (block b -> (row group, direction)
  // slot b & 7, workgroup b >> 3: one XCD per slot under round-robin dispatch)
  const int d = p.xpd ? (blockIdx.x & 7) % dirs : blockIdx.x % dirs;
  const int g = p.xpd ? (blockIdx.x >> 3) : (blockIdx.x / dirs) % NWG;
  const int grp = p.xpd ? (blockIdx.x & 7) / dirs : blockIdx.x / (dirs * NWG);
  if (g >= NWG || grp >= p.rg) return;
  const int N = p.N, T = p.T, n0 = grp * p.gs, nend = min(N, n0 + p.gs);
  const int u0 = g * U;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const long ldy = (long)dirs * H, ldg = (long)dirs * NW * H;
  constexpr long XG = 2L * KB * NP * 16 * 32;  // halves per row group's image of a step (dirs <= 2)
  const long XS = XG * p.rg;                    // halves per step image
  float *red = smem;                                                       // [NWV][16][RP]
  // [NP][16][U], 16-B aligned.  Offset arithmetic on smem only: a pointer
  // rounded through an integer loses the LDS address space, and the staging
  // reads and writes became FLAT instructions (counted in vmcnt, so the
  // publish waited for every store of the step still in flight)
  constexpr int RPR = (U % 16 == 0 && NW <= 4 && 4 * U > RP) ? 4 * U : RP;  // red floats per (wave, row)
  constexpr int kStgOff = (NWV * 16 * RPR + 3 + 3) / 4 * 4;
  AT *stg = reinterpret_cast<AT *>(smem + kStgOff);
  // IO waves: the G rows of step k in slot k & 7, [8][NW][16 U] floats,
  // filled by LDS-DMA p.gla (3 or 7) steps ahead
  float *ginl = smem + kStgOff + (NP * 16 * U + 7) / 8 * 4;  // 16-B aligned
  float *outl = ginl + 8 * NW * 16 * U;  // (IO_OUT) [2][NW + 2][16 U]
  const float *Wd = p.w + d * p.pl_stride;
  const float *R = Wd + p.r_off;
  AT *xch = reinterpret_cast<AT *>(p.xch);
  if (tid == 0) bad_lds = 0;
  // ---- R slice -> B fragments: B[k][c] = R[q*H + u0 + u][k], c = q*U + u ----
  auto rrow = [&](int c) -> const float * {
    const int q = c / U, u = c - q * U;
    return R + (long)(q * H + u0 + u) * H;
  };
  int sB = 0, sOut = 0;
  if constexpr (!BF) {
    float mx = 0.f;
#pragma unroll
    for (int ct = 0; ct < CT; ct++) {
      const int c = ct * 16 + fr;
      if (c < NC) {
        const float *rr = rrow(c);
#pragma unroll
        for (int i = 0; i < KBW; i++) {
          const int kb = (!IOW || w < CW) ? w + CW * i : KB;
          if (kb < KB) {
#pragma unroll
            for (int j = 0; j < 8; j++) mx = fmaxf(mx, fabsf(rr[kb * 32 + fq * 8 + j]));
          }
        }
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    if (lane == 0) wmax[w] = mx;
    __syncthreads();
    float m4 = wmax[0];
#pragma unroll
    for (int i = 1; i < NWV; i++) m4 = fmaxf(m4, wmax[i]);
    sB = split_exp(m4);
    sOut = -(sB + 14);
  }
  AV bhi[CT][KBW], blo[BF ? 1 : CT][BF ? 1 : KBW];
#pragma unroll
  for (int ct = 0; ct < CT; ct++) {
    const int c = ct * 16 + fr;
#pragma unroll
    for (int i = 0; i < KBW; i++) {
      const int kb = (!IOW || w < CW) ? w + CW * i : KB;
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const float v = (c < NC && kb < KB) ? rrow(c)[kb * 32 + fq * 8 + j] : 0.f;
        if constexpr (BF) {
          bhi[ct][i][j] = (__bf16)v;
        } else {
          _Float16 h, l;
          split16(ldexpf(v, sB), h, l);
          bhi[ct][i][j] = h;
          blo[ct][i][j] = l;
        }
      }
    }
  }
  // ---- per-element state: thread tid <-> (row n0 + en, unit u0 + eu) ----
  const bool has_e = tid < 16 * U;
  const int en = tid / U, eu = tid - en * U;
  const int n = n0 + en;
  const bool live = has_e && n < nend;
  float cst = 0.f, hpv = 0.f, cnew = 0.f, hval = 0.f;
  float gin[NW], gnx[NW], bR[NW], act[NW];
#pragma unroll
  for (int q = 0; q < NW; q++) {
    gin[q] = gnx[q] = act[q] = 0.f;
    bR[q] = (MODE == kGru && has_e) ? Wd[p.bR_off + q * H + u0 + eu] : 0.f;
  }
  auto gin_load = [&](int t, float (&dst)[NW]) {
    if (!live) return;
#pragma unroll
    for (int q = 0; q < NW; q++) dst[q] = p.G[((long)t * N + n) * ldg + (long)d * NW * H + q * H + u0 + eu];
  };
  // bf16_io: the step's h (stg, bf16 [16][U]) as packed rows and columns
  auto y_pk_store = [&](int tt) {
    if constexpr (BF) {
      constexpr int RCH = U / 8;
      const long f0 = (long)tt * N + n0;
      const int i = tid;
      if (i < 16 * RCH) {
        const int rn = i / RCH, ch = i - rn * RCH;
        if (n0 + rn < nend)
          *reinterpret_cast<u32x4 *>(p.yr + (f0 + rn) * ldy + (long)d * H + u0 + ch * 8) =
              *reinterpret_cast<const u32x4 *>(stg + rn * U + ch * 8);
      } else if (i < 16 * RCH + 2 * U) {
        const int col = (i - 16 * RCH) >> 1, half = (i - 16 * RCH) & 1, r0 = half * 8;
        __bf16 *dst = p.yc + ((long)d * H + u0 + col) * p.kbt64 + f0 + r0;
        if ((N % 8 == 0) && (n0 % 8 == 0) && n0 + r0 + 8 <= nend) {
          bf16x8 v;
#pragma unroll
          for (int j = 0; j < 8; j++) v[j] = stg[(r0 + j) * U + col];
          *reinterpret_cast<bf16x8 *>(dst) = v;
        } else {
          for (int j = 0; j < 8; j++)
            if (n0 + r0 + j < nend) dst[j] = stg[(r0 + j) * U + col];
        }
      }
    }
  };
  auto out_store = [&](int t) {  // row-major y, activations (in place of G), aux of step t
    if (!live) return;
    if (p.ysc1) __hip_atomic_store(p.y + ((long)t * N + n) * ldy + (long)d * H + u0 + eu, hval, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);  // read by other XCDs during this kernel
    else p.y[((long)t * N + n) * ldy + (long)d * H + u0 + eu] = hval;
    const long grow = ((long)t * N + n) * ldg + (long)d * NW * H + u0 + eu;
#pragma unroll
    for (int q = 0; q < NW; q++) p.G[grow + q * H] = act[q];
    p.aux[((long)t * N + n) * ldy + (long)d * H + u0 + eu] = cnew;
  };
  // IO waves: thread tid - 64 CW <-> element (ion, iou); G of step k into
  // ginl[k & 1] before step k's K-reduction barrier
  const int iot = tid - 64 * CW, ion = iot / U, iou = iot - ion * U;
  const bool io_live = IOW && w >= CW && n0 + ion < nend;
  // G row of forward-order step kk of this lane's element into slot kk & 7
  // by LDS-DMA (lane l of IO wave v writes element 64 v + l); NW DMAs per
  // call whatever kk, so that the waits can count them (rows past N and
  // steps past T read a valid row and are never used)
  auto io_dma = [&](int kk) {
    const int tt = d == 0 ? min(kk, T - 1) : max(T - 1 - kk, 0);
    const long gr = ((long)tt * N + n0 + (io_live ? ion : 0)) * ldg + (long)d * NW * H + u0 + iou;
#pragma unroll
    for (int q = 0; q < NW; q++) {
      const unsigned dst = __builtin_amdgcn_readfirstlane(
          (unsigned)reinterpret_cast<uintptr_t>(ginl + ((kk & 7) * NW + q) * 16 * U + (w - CW) * 64));
      dma_lds_dword(p.G + gr + q * H, dst);
    }
  };
  auto io_out = [&](int kk) {  // row-major outputs of step kk from outl[kk & 1]
    if (!io_live) return;
    const int tt = d == 0 ? kk : T - 1 - kk;
    const float *o = outl + (long)(kk & 1) * (NW + 2) * 16 * U + iot;
    const long yrow = ((long)tt * N + n0 + ion) * ldy + (long)d * H + u0 + iou;
    const long grow = ((long)tt * N + n0 + ion) * ldg + (long)d * NW * H + u0 + iou;
    p.y[yrow] = o[0];
#pragma unroll
    for (int q = 0; q < NW; q++) p.G[grow + q * H] = o[(1 + q) * 16 * U];
    p.aux[yrow] = o[(NW + 1) * 16 * U];
  };
  // the IO waves' wait for step k + 1's G: at most (gla - 1) * NW DMAs (the
  // steps after it) still in flight
  const bool gla7 = p.gla == 7;
  auto io_wait = [&]() {
    if (gla7) {
      if constexpr (NW == 4) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
    } else {
      if constexpr (NW == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    }
  };
  if constexpr (IOW) {
    if (w >= CW) {  // steps 0 .. gla - 1; step 0's in place before the loop's first barrier
      for (int kk = 0; kk < (gla7 ? 7 : 3); kk++) io_dma(kk);
      io_wait();
    }
    __syncthreads();
  } else {
    gin_load(d == 0 ? 0 : T - 1, gin);
  }
  int bad = 0;
  unsigned *myflag = flag6(p, grp, d, g, NWG);
  // XCD-pinned (p.xpd): the hand-off goes through a ring of p.ring step images
  // after the T per-step images, kept in the XCD's L2 (plain stores, workgroup-
  // scope flags) when probe6 finds the direction's workgroups on one XCD; a
  // streamed projection on the other XCDs reads the per-step images, written
  // through (sc1) behind the next step's hand-off loads, and follows sc1
  // copies of the epochs 256 lines on: gflag = k in step k's load phase
  // (step k - 1's signal drained step k - 2's copy), T + 1 at exit -- "epoch
  // - 2 = last step out" as the unpinned flags
  // (aggregated over the direction's workgroups by workgroup 0, as in
  // rnn_bwd_rec6: agg_flag6 = k after the K-reduction barrier of step k, by
  // which every producer's signal of step k - 1 drained its copy of step k - 2)
  // (compiled into the IO-wave variant only, the one chain_ok lets stream
  // off a pinned producer: the dead code of it in the other variants changed
  // their schedules -- U = 32 forward 3.19 -> 4.0 us/step at configs[2])
  const bool fcopy = IOW && p.xpd && p.fcopy;
  // y rows streamed (p.ysc1): step m's y goes out in step m + 1, behind that
  // step's hand-off loads, so it has landed once the workgroup publishes step
  // m + 2; workgroup 0 has every producer's step k - 1 image in step k, so
  // gflag = k there means rows of steps <= k - 3 are out ("epoch s + 3" as
  // the backward's rows), T + 2 at exit
  unsigned *gflag = ((fcopy || p.ysc1) && g == 0) ? agg_flag6(p, grp, d) : nullptr;
  if (tid == 0) {  // (the side launches' residency gate: beside_recurrence)
    if (p.xpd) atomicOr(p.flags + kXcdWord, 1u << xcc_id());
    atomicAdd(p.flags + kResWord, 1u);
  }
  if (tid == 0) loc_lds = 0;
  const int local = (p.xpd && p.allow_local) ? probe6(p, grp, d, g, NWG, bad, &bad_lds, &loc_lds) : 0;
  if (trc_ && tid == 0) trc_[9] = (unsigned long long)(local + 1);  // step 0, slot 9
  const long rbase = (long)T * XS;  // ring slots (p.ring > 0)
  // Self-tagged hand-off (as rnn_bwd_rec6): every fp16 half of step k's h
  // image carries ((k >> 1) & 1) in its LSB (hi's change is taken up by lo,
  // lo's own LSB costs 2^-21 of |h| at most); the consumers poll the image
  // words themselves: no drain, no flag.  Split-fp16 without IO waves, no
  // write-through copy for a streamed projection, ring of two L2 images set
  // to tag 1 before the launch.
  const bool dtag = !BF && !IOW && !fcopy && p.dtag && local && p.ring == 2;
  // the published 16 B of h: live across the whole loop (used after it), so
  // that no other value of the step is allocated to the data registers of the
  // write-through copy still in flight (gfx9 waits for a store's completion
  // before its data VGPRs are overwritten)
  u32x4 pv = u32x4{0u, 0u, 0u, 0u};
  // the per-step images as one loop-invariant buffer (chain_ok: T XS halves < 2 GB)
  const auto crs = rsrc(xch, fcopy ? (unsigned)(T * XS * sizeof(AT)) : 0u);
  // publish geometry: store thread s < NP * 16 * CH: part = s / (16 CH), row, chunk
  const int sp = tid / (16 * CH), sn = (tid / CH) % 16, sch = tid % CH;
  const int kb0 = u0 >> 5, koff = (u0 & 31) + sch * 8;
  // rows past N (a group of fewer than 16 sequences) are neither loaded nor stored
  // (STK: lanes fr >= 8 load the lo part of row fr - 8)
  const bool arow_live = n0 + (STK ? (fr & 7) : fr) < nend;
  // per-wave wait: the producers of the k blocks this wave loads (32 / U per block)
  int wprod = -1;
  {
    constexpr int PPK = 32 / U;
    const int i = lane / PPK, kb = (!IOW || w < CW) ? w + CW * i : KB;
    if (i < KBW && kb < KB) wprod = kb * PPK + lane % PPK;
  }
  const long gimg = (long)grp * XG;
  const bool pub = tid < NP * 16 * CH && n0 + sn < nend;  // a publishing thread: 16 B of h
  const long po = gimg + ((((long)d * KB + kb0) * NP + sp) * 16 + sn) * 32 + koff;
  int t_prev = -1;
  for (int k = 0; k < T && !bad; k++) {
    const int t = d == 0 ? k : T - 1 - k, tp = d == 0 ? t - 1 : t + 1;
    floatx4 acc[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ct++) acc[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
    REC_TRACE(k, 0);
    if (k > 0 && (!IOW || w < CW)) {
      if (dtag) {
        // self-tagged: the poll below is the wait
      } else {
        if (!wave_wait_prod(flag6(p, grp, d, 0, NWG), wprod, (unsigned)(k + 1), p.err, &bad_lds, p.poll_sleep)) bad = 1;
      }
      REC_TRACE(k, 1);
      const auto rs = rsrc(xch + (p.ring ? rbase + (long)((k - 1) & 1) * XS : (long)tp * XS),
                           (unsigned)(XS * sizeof(AT)));
      u32x4 ah[KBW], al[KBW];
      unsigned aoff[KBW];
      // unconditional loads (rows past N and k blocks past KB at an offset
      // past the buffer: the hardware returns zeros), so that the compiler
      // counts them exactly and the first MFMAs wait for their own loads only
#pragma unroll
      for (int i = 0; i < KBW; i++) {
        const int kb = w + CW * i;
        const long o = STK ? gimg + ((((long)d * KB + kb) * NP + (fr >> 3)) * 16 + (fr & 7)) * 32 + fq * 8
                           : gimg + ((((long)d * KB + kb) * NP) * 16 + fr) * 32 + fq * 8;
        const unsigned off = (kb < KB && arow_live) ? (unsigned)(o * sizeof(AT)) : 0x7fff0000u;
        aoff[i] = off;
        ah[i] = ld_sc1(rs, off);
        if constexpr (!BF && !STK) al[i] = ld_sc1(rs, off + 16 * 32 * sizeof(AT));
      }
      if constexpr (!BF) {
        if (dtag) {
          // every half of step k - 1 carries ((k - 1) >> 1) & 1 in its LSB
          // (bits 0 and 16 of a word; 4-B words are single-copy atomic); a
          // chunk still holding step k - 3's halves is loaded again
          const unsigned want = ((unsigned)((k - 1) >> 1) & 1u) * 0x00010001u;
          // (rows past N and k blocks past KB: zeros from past the buffer, no tag)
          const bool any_live = arow_live && w < KB;
          auto ready = [&]() {
            unsigned bad4 = 0u;
#pragma unroll
            for (int i = 0; i < KBW; i++) {
              if (w + CW * i < KB) {
                bad4 |= (ah[i][0] ^ want) | (ah[i][1] ^ want) | (ah[i][2] ^ want) | (ah[i][3] ^ want);
                if constexpr (!STK) bad4 |= (al[i][0] ^ want) | (al[i][1] ^ want) | (al[i][2] ^ want) | (al[i][3] ^ want);
              }
            }
            return !any_live || (bad4 & 0x00010001u) == 0u;
          };
          int spins = 0;
          while (!__all(ready())) {  // (not all there yet: the wave loads all its chunks again)
            if (++spins > kSpinLimit ||
                ((spins & 255) == 0 &&
                 __builtin_amdgcn_readfirstlane(__hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)))) {
              bad = 1;
              if (lane == 0) bad_lds = 1;
              break;
            }
            if (p.poll_sleep) __builtin_amdgcn_s_sleep(1);
            asm volatile("" ::: "memory");
#pragma unroll
            for (int i = 0; i < KBW; i++) {
              ah[i] = ld_sc1(rs, aoff[i]);
              if constexpr (!BF && !STK) al[i] = ld_sc1(rs, aoff[i] + 16 * 32 * sizeof(AT));
            }
          }
        }
      }
      // all hand-off loads in flight before the first MFMA waits: without
      // this the scheduler (U = 32) issued the second k block's loads only
      // after the first block's MFMAs, one more L2 round trip per step
      __builtin_amdgcn_sched_barrier(0);
      // the streamed projection's write-through copy of the previous step's
      // image (pv still holds it), issued behind this step's hand-off loads:
      // gfx9 counts stores and loads in one vmcnt, so a write-through store
      // in flight at the next flag poll would hold up that poll; here the
      // waits for the loads ahead of it do not cover it, and this step's
      // signal drains it (the next step publishes its epoch)
      // (every lane of every wave issues it -- non-publishing lanes at an
      // offset past the buffer, which the hardware drops -- so that no
      // branch makes the compiler's wait counts conservative)
      // (unconditional: without a consumer crs covers 0 bytes and the store is dropped)
      __builtin_amdgcn_raw_buffer_store_b128(pv, crs, pub ? (int)(po * sizeof(AT)) : 0x7ffffff0,
                                             fcopy ? (int)(tp * XS * sizeof(AT)) : 0, 16);

#pragma unroll
      for (int i = 0; i < KBW; i++) {
        if (w + CW * i < KB) {
          const AV a0 = __builtin_bit_cast(AV, ah[i]);
          if constexpr (BF) {
#pragma unroll
            for (int ct = 0; ct < CT; ct++) acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bhi[ct][i], acc[ct], 0, 0, 0);
          } else if constexpr (STK) {
#pragma unroll
            for (int ct = 0; ct < CT; ct++) acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, bhi[ct][i], acc[ct], 0, 0, 0);
#pragma unroll
            for (int ct = 0; ct < CT; ct++) acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, blo[ct][i], acc[ct], 0, 0, 0);
          } else {
            const AV a1 = __builtin_bit_cast(AV, al[i]);
#pragma unroll
            for (int ct = 0; ct < CT; ct++) acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, bhi[ct][i], acc[ct], 0, 0, 0);
#pragma unroll
            for (int ct = 0; ct < CT; ct++) acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, blo[ct][i], acc[ct], 0, 0, 0);
#pragma unroll
            for (int ct = 0; ct < CT; ct++) acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, bhi[ct][i], acc[ct], 0, 0, 0);
          }
        }
      }
    }
    asm volatile("" ::: "memory");
    // behind the hand-off loads: last step's row-major outputs, next step's input projection
    if (!IO_OUT && t_prev >= 0) out_store(t_prev);
    // (stg still holds step t_prev's h: the cell phase below rewrites it)
    if (BF && p.yr && t_prev >= 0) y_pk_store(t_prev);
    if (!IOW && k + 1 < T) gin_load(d == 0 ? t + 1 : t - 1, gnx);
    // K partials through LDS.  U % 16 == 0: column ct * 16 + fr of the
    // tile is gate ct / (U / 16) of unit (ct % (U / 16)) * 16 + fr, so a lane
    // holds every gate of its (row, unit) elements: one float4 per (wave,
    // row, unit) [NWV][16][U][4], and a cell thread sums NWV float4 reads
    // (4x fewer LDS instructions than one float per gate)
    constexpr bool RED4 = U % 16 == 0 && NW <= 4;
    if constexpr (STK) {  // rows 8..15 hold the lo parts' products: fold them into rows 0..7
#pragma unroll
      for (int ct = 0; ct < CT; ct++)
#pragma unroll
        for (int i = 0; i < 4; i++) acc[ct][i] = fold_rows8(acc[ct][i]);
    }
    if constexpr (RED4) {
      constexpr int SU = U / 16;
      if (!IOW || w < CW) {
#pragma unroll
        for (int su = 0; su < SU; su++)
#pragma unroll
          for (int i = 0; i < 4; i++) {
            floatx4 v4 = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int q = 0; q < NW; q++) v4[q] = acc[q * SU + su][i];
            st4(red + (((long)(w * 16 + fq * 4 + i) * U + su * 16 + fr) << 2), v4);
          }
      }
    } else {
#pragma unroll
      for (int ct = 0; ct < CT; ct++)
#pragma unroll
        for (int i = 0; i < 4; i++) red[(w * 16 + fq * 4 + i) * RP + ct * 16 + fr] = acc[ct][i];
    }
    lds_barrier<IOW>();
    if (bad_lds) bad = 1;
    // the aggregated epoch (before the signal: a write-through flag store
    // left in flight there would hold up the next step's first flag poll)
    if (gflag && k > 0 && tid == 0) __hip_atomic_store(gflag, (unsigned)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    REC_TRACE(k, 3);
    if (has_e) {
      float rh[NW];
      if constexpr (RED4) {
        floatx4 sm = *reinterpret_cast<const floatx4 *>(red + (((long)en * U + eu) << 2));  // fixed order
#pragma unroll
        for (int v = 1; v < CW; v++) sm += *reinterpret_cast<const floatx4 *>(red + (((long)(v * 16 + en) * U + eu) << 2));
        if constexpr (IOW) {  // this step's G row, put there by the IO waves
#pragma unroll
          for (int q = 0; q < NW; q++) gin[q] = ginl[((k & 7) * NW + q) * 16 * U + tid];
        }
#pragma unroll
        for (int q = 0; q < NW; q++) rh[q] = BF ? sm[q] : ldexpf(sm[q], sOut);
      } else {
#pragma unroll
        for (int q = 0; q < NW; q++) {
          const int c = q * U + eu;
          float sm = red[(0 * 16 + en) * RP + c];  // the waves' K partials in a fixed order
#pragma unroll
          for (int v = 1; v < NWV; v++) sm += red[(v * 16 + en) * RP + c];
          rh[q] = BF ? sm : ldexpf(sm, sOut);
        }
      }
      float h;
      if (MODE == kLstm) {
        act[0] = fsigm(gin[0] + rh[0]);
        act[1] = fsigm(gin[1] + rh[1]);
        act[2] = ftanh(gin[2] + rh[2]);
        act[3] = fsigm(gin[3] + rh[3]);
        cst = act[1] * cst + act[0] * act[2];
        cnew = cst;
        h = act[3] * ftanh(cst);
      } else {
        act[0] = fsigm(gin[0] + rh[0] + bR[0]);
        act[1] = fsigm(gin[1] + rh[1] + bR[1]);
        cnew = rh[2] + bR[2];
        act[2] = ftanh(gin[2] + act[0] * cnew);
        h = (1.f - act[1]) * act[2] + act[1] * hpv;
        hpv = h;
      }
      if (!live) h = 0.f;
      hval = h;
      if constexpr (!IOW) {
        // the next step's input projection (loaded behind this step's
        // hand-off loads) moves in here
#pragma unroll
        for (int q = 0; q < NW; q++) gin[q] = gnx[q];
      }
      if constexpr (IO_OUT) {  // outputs for the IO waves (stored during the next step)
        float *o = outl + (long)(k & 1) * (NW + 2) * 16 * U + tid;
        o[0] = h;
#pragma unroll
        for (int q = 0; q < NW; q++) o[(1 + q) * 16 * U] = act[q];
        o[(NW + 1) * 16 * U] = cnew;
      }

      if constexpr (BF) {
        stg[en * U + eu] = (__bf16)h;
      } else {
        _Float16 hh, hl;
        if (!IOW) {  // hi's LSB := tag, lo takes up the change, then lo's LSB := tag
          // (in every mode a self-tagged launch may take: pinned and unpinned
          // runs stay bit-identical)
          const unsigned short tgh = (unsigned short)((k >> 1) & 1);
          const float x = h * 16384.f;
          hh = __builtin_bit_cast(_Float16, (unsigned short)((__builtin_bit_cast(unsigned short, (_Float16)x) & 0xFFFEu) | tgh));
          hl = __builtin_bit_cast(_Float16, (unsigned short)((__builtin_bit_cast(unsigned short, (_Float16)(x - (float)hh)) & 0xFFFEu) | tgh));
        } else {
          split16(h * 16384.f, hh, hl);
        }
        stg[en * U + eu] = hh;
        stg[(16 + en) * U + eu] = hl;
      }
    }
    if (IOW && w >= CW) {
      // IO waves, while the cell threads work: step k + 1's G (loaded during
      // step k - 1) into its slot -- read by the cell threads after the next
      // K-reduction barrier; the slot's step k - 1 readers passed the
      // barrier below last step -- then step k + 2's loads, then the
      // row-major outputs of step k - 1 (written before the last barrier;
      // their slot is rewritten after the next K-reduction barrier)
      {
        // step k + gla's G into slot (k + gla) & 7 (gla <= 7: last read by the
        // cell threads of step k - 1 at the latest, before the last barrier),
        // then wait for step k + 1's: in place before the barrier below,
        // gla - 1 steps after it was asked for
        io_dma(k + (gla7 ? 7 : 3));
        io_wait();
      }
      if (IO_OUT && k > 0) io_out(k - 1);
    }
    lds_barrier<IOW>();
    if (pub) {
      pv = *reinterpret_cast<const u32x4 *>(stg + (sp * 16 + sn) * U + sch * 8);
      const auto ro = rsrc(xch + (p.ring ? rbase + (long)(k & 1) * XS : (long)t * XS), (unsigned)(XS * sizeof(AT)));
      // local: plain stores stay in the XCD's L2 for the consumers' sc1 loads
      if (local) __builtin_amdgcn_raw_buffer_store_b128(pv, ro, (int)(po * sizeof(AT)), 0, 0);
      else __builtin_amdgcn_raw_buffer_store_b128(pv, ro, (int)(po * sizeof(AT)), 0, 16);
    }
    REC_TRACE(k, 7);
    if constexpr (NP * 16 * CH <= 64) {
      // one publishing wave (wave 0 stores the whole h part): it drains its
      // own stores and raises the flag, no workgroup barrier.  The other
      // waves go on to the next step's wait: their reads of red and stg this
      // step all came before the barrier above, and the next writes of either
      // follow the next K-reduction barrier, which wave 0 reaches only after
      // its stg read
      if (w == 0 && !dtag) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
          if (local) __hip_atomic_store(myflag, (unsigned)(k + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          else __hip_atomic_store(myflag, (unsigned)(k + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    } else if (!dtag) {
      signal_epoch(myflag, (unsigned)(k + 2), local);
    }
    REC_TRACE(k, 4);
    t_prev = t;
    REC_TRACE(k, 5);
  }
  if (IOW && w >= CW) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the IO waves' DMAs (ahead of T) land
  if (t_prev >= 0 && !bad) {
    if (BF && p.yr) y_pk_store(t_prev);
    if constexpr (IO_OUT) {
      if (w >= CW) io_out(T - 1);  // outl of the last step: written before the loop's last barrier
    } else {
      out_store(t_prev);
    }
  }
  if ((fcopy || p.ysc1) && !bad) {  // the last step's copy / rows, then (workgroup 0) every producer's, then the epoch
    if (fcopy && pub)
      __builtin_amdgcn_raw_buffer_store_b128(pv, rsrc(xch + (long)t_prev * XS, (unsigned)(XS * sizeof(AT))),
                                             (int)(po * sizeof(AT)), 0, 16);
    signal_epoch(myflag, (unsigned)(T + 2), local);
    if (gflag) {
      wait_flags6(flag6(p, grp, d, 0, NWG), NWG, (unsigned)(T + 2), p.err, bad, &bad_lds, p.poll_sleep);
      if (!bad && tid == 0)
        __hip_atomic_store(gflag, (unsigned)(fcopy ? T + 1 : T + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("" ::"v"(pv));
  if (bad && tid == 0) atomicOr(p.err, 1u);
}

template <typename F>
static void set_lds(F f, size_t bytes) {
  static size_t done[8] = {0};
  (void)done;
  (void)hipFuncSetAttribute(reinterpret_cast<const void *>(f), hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)bytes);
}

template <int MODE, int RT>
static void launch_one(bool fwd, const RecParams &p, dim3 grid, size_t lds, hipStream_t s, int ver) {
  if (ver == 4) {
    if (fwd) {
      set_lds(rnn_fwd_rec4<MODE, RT>, lds);
      hipLaunchKernelGGL((rnn_fwd_rec4<MODE, RT>), grid, dim3(NT), lds, s, p);
    } else {
      set_lds(rnn_bwd_rec4<MODE, RT>, lds);
      hipLaunchKernelGGL((rnn_bwd_rec4<MODE, RT>), grid, dim3(NT), lds, s, p);
    }
    return;
  }
  if (fwd) {
    set_lds(rnn_fwd_rec<MODE, RT>, lds);
    hipLaunchKernelGGL((rnn_fwd_rec<MODE, RT>), grid, dim3(NT), lds, s, p);
  } else {
    set_lds(rnn_bwd_rec<MODE, RT>, lds);
    hipLaunchKernelGGL((rnn_bwd_rec<MODE, RT>), grid, dim3(NT), lds, s, p);
  }
}
template <int MODE>
static void launch_mode(bool fwd, const RecParams &p, dim3 grid, size_t lds, hipStream_t s, int ver) {
  switch (p.Npad / 16) {
    case 1: launch_one<MODE, 1>(fwd, p, grid, lds, s, ver); break;
    case 2: launch_one<MODE, 2>(fwd, p, grid, lds, s, ver); break;
    case 3: launch_one<MODE, 3>(fwd, p, grid, lds, s, ver); break;
    default: launch_one<MODE, 4>(fwd, p, grid, lds, s, ver); break;
  }
}
// v6 shapes that compile: H in {256, 320, 512, 1024}; U in {8, 16} at 256
// threads, U = 32 at 512 threads (H / (16 * waves) output tiles per wave and
// H / U producers in groups of 512 / (4 U) for the backward)
template <int U, int H, int NTH>
constexpr bool v6_shape_ok() {
  return (NTH == (U == 32 ? 512 : 256) || (U == 16 && (NTH == 512 || NTH == 1024) && H == 512)) && H % (16 * (NTH / 64)) == 0 &&
         (H / U) % (NTH / (4 * U)) == 0;
}
// rec6_scratch_bytes: launch6 with this set names the kernel it would launch
// (its private segment size lands here) instead of launching it
thread_local size_t *g_rec6_probe = nullptr;
static size_t kernel_scratch(const void *f) {
  hipFuncAttributes a{};
  KCTC_HIP_CHECK(hipFuncGetAttributes(&a, f));
  return a.localSizeBytes;
}
template <int MODE, int U, int H, int NTH, int P>
static void launch6_shape(bool fwd, const RecParams &p, dim3 grid, size_t lds, hipStream_t s) {
  if constexpr (v6_shape_ok<U, H, NTH>()) {
    if (g_rec6_probe) {
      if (fwd) *g_rec6_probe = kernel_scratch(reinterpret_cast<const void *>(rnn_fwd_rec6<MODE, U, H, NTH, P>));
      else if constexpr ((P & 4) == 0)
        *g_rec6_probe = kernel_scratch(reinterpret_cast<const void *>(rnn_bwd_rec6<MODE, U, H, NTH, P>));
      return;
    }
    if (fwd) {
      set_lds(rnn_fwd_rec6<MODE, U, H, NTH, P>, lds);
      hipLaunchKernelGGL((rnn_fwd_rec6<MODE, U, H, NTH, P>), grid, dim3(NTH), lds, s, p);
    } else if constexpr ((P & 4) == 0) {
      set_lds(rnn_bwd_rec6<MODE, U, H, NTH, P>, lds);
      hipLaunchKernelGGL((rnn_bwd_rec6<MODE, U, H, NTH, P>), grid, dim3(NTH), lds, s, p);
    } else {
      throw std::logic_error("v6 recurrence: IO waves are a forward variant");
    }
  } else {
    throw std::logic_error("v6 recurrence: shape not compiled");
  }
}
template <int MODE, int U, int NTH, int P>
static void launch6_h(bool fwd, const RecParams &p, dim3 grid, size_t lds, hipStream_t s) {
  switch (p.H) {
    case 256: launch6_shape<MODE, U, 256, NTH, P>(fwd, p, grid, lds, s); break;
    case 320: launch6_shape<MODE, U, 320, NTH, P>(fwd, p, grid, lds, s); break;
    case 512: launch6_shape<MODE, U, 512, NTH, P>(fwd, p, grid, lds, s); break;
    case 1024: launch6_shape<MODE, U, 1024, NTH, P>(fwd, p, grid, lds, s); break;
    default: throw std::logic_error("v6 recurrence: H not compiled");
  }
}
static int env_int(const char *name, int dflt);
template <int MODE, int P>
static void launch6_u(bool fwd, int nth, const RecParams &p, dim3 grid, size_t lds, hipStream_t s) {
  switch (p.U) {
    case 8: launch6_h<MODE, 8, 256, P>(fwd, p, grid, lds, s); break;
    case 16:
      if (nth == 1024) launch6_h<MODE, 16, 1024, P>(fwd, p, grid, lds, s);
      else if (nth == 512) {
        // row groups of <= 8 sequences: hi / lo stacked in one MFMA operand
        // (all four products: equally accurate or better), on by default in
        // both directions: the stacked forward (one A load per k block, 2/3
        // of the MFMAs) runs 1.76 us/step against 2.05 for the IO-wave
        // forward (round 4); the transposed stacked backward with its DPP row
        // fold 1.91 against 2.43 (round 5).  KCTC_STK_FWD (forward; KCTC_STK
        // for both)
        const int stk = fwd ? env_int("KCTC_STK_FWD", env_int("KCTC_STK", 1)) : env_int("KCTC_STK", 1);
        if constexpr (P == kPrecX3) {
          if (p.gs <= 8 && stk) {
            launch6_h<MODE, 16, 512, kPrecX3S>(fwd, p, grid, lds, s);
            break;
          }
        }
        // forward with IO waves (the G loads off the hand-off waves)
        if constexpr (MODE == kLstm || MODE == kGru) {
          if (fwd) {
            launch6_h<MODE, 16, 512, P | 4>(fwd, p, grid, lds, s);
            break;
          }
        }
        launch6_h<MODE, 16, 512, P>(fwd, p, grid, lds, s);
      } else {
        launch6_h<MODE, 16, 256, P>(fwd, p, grid, lds, s);
      }
      break;
    default: launch6_h<MODE, 32, 512, P>(fwd, p, grid, lds, s); break;
  }
}
static void launch6(bool fwd, int mode, int prec, int nth, const RecParams &p, dim3 grid, size_t lds,
                    hipStream_t s) {
  if (mode == kLstm) {
    if (prec == kPrecBf16) launch6_u<kLstm, kPrecBf16>(fwd, nth, p, grid, lds, s);
    else launch6_u<kLstm, kPrecX3>(fwd, nth, p, grid, lds, s);
  } else {
    if (prec == kPrecBf16) launch6_u<kGru, kPrecBf16>(fwd, nth, p, grid, lds, s);
    else launch6_u<kGru, kPrecX3>(fwd, nth, p, grid, lds, s);
  }
}
static void launch_rec(bool fwd, int mode, const RecParams &p, dim3 grid, size_t lds, hipStream_t s,
                       int ver) {
  switch (mode) {
    case kLstm: launch_mode<kLstm>(fwd, p, grid, lds, s, ver); break;
    case kGru: launch_mode<kGru>(fwd, p, grid, lds, s, ver); break;
    case kRelu: launch_mode<kRelu>(fwd, p, grid, lds, s, ver); break;
    default: launch_mode<kTanh>(fwd, p, grid, lds, s, ver); break;
  }
}

// KCTC_REC_TRACE=<dir>: trace the first forward and the first backward
// recurrence launch of the process into <dir>/rec_{fwd,bwd}.bin
// (int32 header {grid, steps, nwg, T, dirs, version, xpd, stride} then [steps][grid][stride] uint64 stamps).
struct RecTrace {
  unsigned long long *dev = nullptr;
  size_t n = 0;
  bool arm(const char *tag, int grid) {
    static bool done_fwd = false, done_bwd = false;
    const char *dir = getenv("KCTC_REC_TRACE");
    if (!dir || !*dir) return false;
    bool &done = tag[0] == 'f' ? done_fwd : done_bwd;
    if (done) return false;
    done = true;
    n = (size_t)kTraceSteps * grid * kTraceStride;
    KCTC_HIP_CHECK(hipMalloc(&dev, n * sizeof(unsigned long long)));
    KCTC_HIP_CHECK(hipMemset(dev, 0, n * sizeof(unsigned long long)));
    return true;
  }
  void dump(const char *tag, hipStream_t s, int grid, int nwg, int T, int dirs, int ver, int xpd = 1) {
    if (!dev) return;
    KCTC_HIP_CHECK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h(n);
    KCTC_HIP_CHECK(hipMemcpy(h.data(), dev, n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    (void)hipFree(dev);
    dev = nullptr;
    std::string path = std::string(getenv("KCTC_REC_TRACE")) + "/rec_" + tag + ".bin";
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) return;
    int hdr[8] = {grid, kTraceSteps, nwg, T, dirs, ver, xpd, kTraceStride};
    fwrite(hdr, sizeof(int), 8, f);
    fwrite(h.data(), sizeof(unsigned long long), n, f);
    fclose(f);
  }
};

static int env_int(const char *name, int dflt) {
  const char *v = getenv(name);
  return v ? atoi(v) : dflt;
}

// pick U (units per workgroup): divides H, multiple of 4, blocks <= 256
static int pick_fwd_u(const RnnDesc &d, int N) {
  const int NW = d.nw();
  auto ok = [&](int U) {
    if (U < 4 || U % 4 || d.H % U || NW * U > 16 * kMaxCT || N * U / 4 > NT) return false;
    if ((long)d.dirs * (d.H / U) > 256) return false;
    const int ncol = (NW * U + 15) / 16 * 16, Npad = (N + 15) / 16 * 16;
    const size_t lds = sizeof(float) * ((size_t)ncol * (d.H + 4) + 4 * (size_t)Npad * ncol);
    return lds <= 160 * 1024;
  };
  // smallest U that keeps every workgroup resident (<= 256 = one per CU):
  // per-step MFMA latency falls with U (measured: U=4 < 8 < 16 on BLSTM-512)
  for (int U : {4, 8, 16})
    if (ok(U)) return U;
  return 0;
}

// v4 (XCD-local): nwg = H/U <= kCusPerXcd workgroups per direction, one XCD each.
constexpr int kCusPerXcd = 32;
static size_t fwd_lds_bytes(const RnnDesc &d, int N, int U) {
  const int ncol = (d.nw() * U + 15) / 16 * 16, Npad = (N + 15) / 16 * 16;
  return sizeof(float) * ((size_t)ncol * (d.H + 4) + 4 * (size_t)Npad * ncol);
}
static size_t bwd_lds_bytes(const RnnDesc &d, int N, int U, int ver = 3) {
  const int Npad = (N + 15) / 16 * 16;
  return sizeof(float) * ((size_t)(ver == 4 ? 16 : U) * (d.nw() * d.H + 4) +
                          std::max(4 * (size_t)Npad * 16, (size_t)2 * N * U * d.nw()));
}
static int rec_version() { return 4; }
// XCD slots one direction spans for U units per workgroup (0: not a v4 shape)
static int v4_xpd(const RnnDesc &d, int U) {
  if (U <= 0 || d.H % U) return 0;
  const int nwg = d.H / U;
  if (nwg % kCusPerXcd) return nwg < kCusPerXcd && d.dirs <= 8 ? 1 : 0;
  const int x = nwg / kCusPerXcd;
  return (x == 1 || x == 2 || x == 4 || x == 8) && x * d.dirs <= 8 ? x : 0;
}
static int pick_fwd_u4(const RnnDesc &d, int N) {
  if (rec_version() != 4 || d.dirs > 8) return 0;
  auto ok = [&](int U) {
    return U >= 4 && U % 4 == 0 && v4_xpd(d, U) && d.nw() * U <= 16 * kMaxCT && N * U <= kMaxEPT * NT &&
           fwd_lds_bytes(d, N, U) <= 160 * 1024;
  };
  // measured on BLSTM-512 N=16 (1 x MI355X): U=8 (2 XCD slots per direction)
  // 44 ms/step of forward recurrence, U=4 48, U=16 58
  for (int U : {8, 16, 4, 32})
    if (ok(U)) return U;
  return 0;
}
static int pick_bwd_u4(const RnnDesc &d, int N) {
  if (rec_version() != 4 || d.dirs > 8) return 0;
  auto ok = [&](int U) {
    return U >= 4 && U <= 16 && U % 4 == 0 && v4_xpd(d, U) && N * U <= kMaxEPT * NT &&
           bwd_lds_bytes(d, N, U, 4) <= 160 * 1024;
  };
  for (int U : {16, 8, 4})
    if (ok(U)) return U;
  return 0;
}

// v6 recurrences (LSTM / GRU): one configuration for a (shape, N):
//   rg   row groups of 16 sequences, each an independent recurrence
//   U    units per workgroup (8, 16 at 256 threads; 32 at 512 threads)
// chosen so that dirs * (H / U) * rg workgroups (one per CU, >= 96 KB LDS
// each) stay within 128 workgroups (half the chip, the rest
// for the GEMMs that overlap the recurrences).  Preference U = 16, then 32,
// then 8 (measured on BLSTM-512 N=16: U=16 34.2 ms/step of forward
// recurrence, U=8 37.1).
// Sequences per v6 row group: 16 (one MFMA row tile), or 8 for 9 <= N <= 32
// -- the batch then runs as ceil(N / 8) independent recurrences side by side,
// each moving half the hand-off rows per step.  Default 8 for N <= 16
// (configs[1]: forward 28.0 -> 27.0, backward 34.2 -> 33.0 ms/step of
// recurrence; the weight GEMMs beside the backward get 64 CUs fewer and take
// twice as long, still hidden).  KCTC_REC_GS sets both directions; a set
// knob applies up to N = 32.  pick6
// falls back to 16 when no workgroup partition fits the groups of 8.
static int v6_group_rows(int N, bool fwd) {
  const int dflt = N <= 16 ? 8 : 16;
  const int want = env_int("KCTC_REC_GS", dflt);
  return (want == 8 && N > 8 && N <= 32) ? 8 : 16;
}
struct V6Cfg {
  int U = 0, nth = 0, rg = 0, gs = 16;
  explicit operator bool() const { return U > 0; }
};
static V6Cfg pick6(const RnnDesc &d, int N, bool fwd, int gs_force = 0) {
  V6Cfg c;
  if (rec_version() != 4) return c;
  if ((d.mode != kLstm && d.mode != kGru) || N <= 0 || N > 64 || d.dirs > 2) return c;
  if (d.H != 256 && d.H != 320 && d.H != 512 && d.H != 1024) return c;
  const int gs = gs_force ? gs_force : v6_group_rows(N, fwd), rg = (N + gs - 1) / gs;
  // never more workgroups than the CUs this process may use (all must be resident)
  const int max_wg = std::min(128, rnn_usable_cus());
  auto ok = [&](int U) {
    const int nth = U == 32 ? 512 : 256, nwv = nth / 64;
    if (d.H % U || d.H % (16 * nwv) || (d.H / U) % (nth / (4 * U))) return false;
    return (long)d.dirs * (d.H / U) * rg <= std::max(max_wg, d.dirs * (d.H / U));  // rg = 1 always fits
  };
  auto take = [&](int U) {
    c.U = U;
    // U = 16 at H = 512 runs 512 threads (K split over 8 waves; measured on
    // BLSTM-512 N=16: forward 31.9 -> 28.4, backward 34.4 -> 32.9 ms/step of
    // recurrence vs 256 threads; 1024 threads 30.5 / 33.5)
    const int want_nth = d.H == 512 ? 512 : 256;
    c.nth = U == 32 ? 512 : (U == 16 && d.H == 512 && (want_nth == 512 || want_nth == 1024)) ? want_nth : 256;
    c.rg = rg;
    c.gs = gs;
    return c;
  };
  for (int U : {16, 32, 8})
    if (ok(U)) {
      // rg = 1 keeps the measured N <= 16 choice even above the budget
      if (rg == 1 || (long)d.dirs * (d.H / U) * rg <= max_wg) return take(U);
    }
  return gs == 8 ? pick6(d, N, fwd, 16) : c;
}
static int pick_fwd_u6(const RnnDesc &d, int N) { return pick6(d, N, true).U; }
static int pick_bwd_u6(const RnnDesc &d, int N) { return pick6(d, N, false).U; }

static size_t fwd6_lds_bytes(const RnnDesc &d, const V6Cfg &c) {
  const int CT = (d.nw() * c.U + 15) / 16, nwv = c.nth / 64, np = d.prec == kPrecBf16 ? 1 : 2;
  const size_t rp = std::max(CT * 16 + 1, 4 * c.U);  // rnn_fwd_rec6's RPR (float4 K partials)
  // + the IO waves' G (and output) slots, for the shape that runs them (launch6_u)
  const bool iow = c.U == 16 && c.nth == 512;
  const size_t b = sizeof(float) * (nwv * 16 * rp + 8) + np * 16 * (size_t)c.U * 2 + 16 +
                   (iow ? sizeof(float) * 16 * c.U * (8 * d.nw() + 2 * (d.nw() + 2)) + 16 + 4 * 64 * 4 : 0);
  return std::max(b, (size_t)96 * 1024);  // one recurrence workgroup per CU
}
static size_t bwd6_lds_bytes(const RnnDesc &d, const V6Cfg &c) {
  const int K = d.nw() * c.U, KB = (K + 31) / 32, AP = KB * 32 + 8;
  const size_t img = (d.prec == kPrecBf16 ? 1 : 2) * 16 * (size_t)AP * 2;
  const size_t red = sizeof(float) * std::max((size_t)c.nth * 4, (size_t)2 * 16 * c.U * d.nw());
  // dGates tile staged for write-through, and (bf16, packed writes) the E tile beside it
  const size_t estg = sizeof(float) * 16 * c.U * d.nw() * (d.prec == kPrecBf16 ? 2 : 1);
  // at least 96 KB so that no other workgroup (a side-stream GEMM block)
  // shares the CU with a recurrence workgroup
  return std::max(img + red + estg, (size_t)96 * 1024);
}

// Per-device exchange pool of the v6 backward: one step image per time step,
// never reused within a launch (T x dirs x nwg x H x Npad floats, 4.2 GB for
// BLSTM-512 N=16 T=2000).  Library-owned so that the components of a network
// share it; launches on one device are ordered through its event.
namespace {
struct XchPool {
  void *p = nullptr;
  size_t bytes = 0;
  hipEvent_t ev = nullptr;
};
std::mutex g_xch_mu;
XchPool g_xch[64];
}  // namespace

static float *xch_acquire(size_t bytes, hipStream_t s) {
  int dev = 0;
  KCTC_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_xch_mu);
  XchPool &x = g_xch[dev & 63];
  if (x.ev) KCTC_HIP_CHECK(hipStreamWaitEvent(s, x.ev, 0));
  if (bytes > x.bytes) {
    if (x.p) {
      KCTC_HIP_CHECK(hipDeviceSynchronize());
      KCTC_HIP_CHECK(hipFree(x.p));
      x.p = nullptr;
    }
    KCTC_HIP_CHECK(hipMalloc(&x.p, bytes));
    x.bytes = bytes;
  }
  return static_cast<float *>(x.p);
}
static void xch_release(hipStream_t s) {
  int dev = 0;
  KCTC_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_xch_mu);
  XchPool &x = g_xch[dev & 63];
  if (!x.ev) KCTC_HIP_CHECK(hipEventCreateWithFlags(&x.ev, hipEventDisableTiming));
  KCTC_HIP_CHECK(hipEventRecord(x.ev, s));
}

static int pick_bwd_u(const RnnDesc &d, int N) {
  const int K = d.nw() * d.H;
  auto ok = [&](int U) {
    if (U < 4 || U % 4 || U > 16 || d.H % U || N * U / 4 > NT) return false;
    if ((long)d.dirs * (d.H / U) > 256) return false;
    const int Npad = (N + 15) / 16 * 16;
    const size_t lds = sizeof(float) * ((size_t)U * (K + 4) + std::max(4 * (size_t)Npad * 16,
                                                                        (size_t)2 * N * U * d.nw()));
    return lds <= 160 * 1024;
  };
  for (int U : {16, 8, 4})
    if (ok(U)) return U;
  return 0;
}

}  // namespace

// ---- launches beside a running recurrence (rnn.h rnn_side_gated) ----
namespace {
// the v6 recurrence this host thread enqueued last, while the host function
// that enqueued it runs (RecScope), and the side streams gated on it
struct RecInFlight {
  const unsigned *res = nullptr;    // its residency word (p.flags + kResWord)
  const unsigned *flags = nullptr;  // its flag area
  unsigned target = 0;              // its workgroups
  hipStream_t gated[4] = {};
  int ngated = 0;
};
thread_local RecInFlight g_rec;
// from a recurrence's launch to the end of the enclosing host call
struct RecScope {
  ~RecScope() { g_rec = RecInFlight{}; }
  void enqueued(const RecParams &p) {
    g_rec = RecInFlight{};
    g_rec.res = p.flags + kResWord;
    g_rec.flags = p.flags;
    g_rec.target = (unsigned)(p.dirs * p.nwg * p.rg);
  }
  void none() { g_rec = RecInFlight{}; }  // (a v3 / v4 recurrence: no side launches)
};
// `side` waits until every workgroup of the recurrence in flight is resident;
// whatever is enqueued on it afterwards may run beside that recurrence
void beside_recurrence(hipStream_t side) {
  if (!g_rec.res) throw std::logic_error("beside_recurrence: no recurrence in flight");
  for (int i = 0; i < g_rec.ngated; i++)
    if (g_rec.gated[i] == side) return;  // (already behind this recurrence's gate)
  if (g_rec.ngated == 4) throw std::logic_error("beside_recurrence: too many side streams");
  rnn_resident_gate(side, g_rec.flags, g_rec.target);
  g_rec.gated[g_rec.ngated++] = side;
}
}  // namespace

thread_local bool g_last_bwd_scratch_free = true;
bool rnn_last_bwd_scratch_free() { return g_last_bwd_scratch_free; }

bool rnn_side_gated(hipStream_t s) {
  if (!g_rec.res) return true;
  for (int i = 0; i < g_rec.ngated; i++)
    if (g_rec.gated[i] == s) return true;
  return false;
}

// ---------------------------------------------------------------------------
// host: forward training
// ---------------------------------------------------------------------------
namespace {
// The recurrence and a GEMM streaming off it must run at the same time, so
// the GEMM's stream forks from the recurrence's stream at an event recorded
// BEFORE the recurrence launch, and the GEMM is enqueued AFTER it: should the
// two streams share a hardware queue, the GEMM then merely runs after the
// recurrence instead of blocking it (its blocks only wait for recurrence flags).
int g_usable_cus = 0, g_comm_cus = 0;

// Does the v6 recurrence of (d, N) run without scratch (no register
// spills)?  Nothing runs beside one that does.  Round 6 first blamed scratch
// for configs[4]'s KCTC_STREAM_ALL hang (the bf16 GRU backward, then 124 B of
// spills per lane, stayed short of its 32 workgroups on one XCD for 0.4 s
// behind the one-wave residency wait of its dx stream); with the spills gone
// it hung the same way: the cause is its 256 VGPRs x 2 waves per SIMD, a
// whole CU's register file, which no workgroup gets on a CU where a gate wave
// sits -- gate_kernel's blocks now leave the recurrence's XCDs
// (tests/test_fullsize_gpu.py cfg4+stream_all).  The scratch
// condition stays as a precaution (no recipe-shape recurrence uses scratch).
bool rec6_scratch_free(const RnnDesc &d, int N, bool fwd) {
  const V6Cfg c6 = pick6(d, N, fwd);
  if (!c6) return false;
  static thread_local std::map<long, bool> memo;
  const int stk = fwd ? env_int("KCTC_STK_FWD", env_int("KCTC_STK", 1)) : env_int("KCTC_STK", 1);
  const long key = ((((long)fwd * 4 + d.mode) * 4 + d.prec) * 64 + c6.U) * 2048 * 2048 + (long)c6.nth * 2048 * 2 +
                   (long)d.H * 2 + (c6.gs <= 8 && stk ? 1 : 0);
  auto it = memo.find(key);
  if (it != memo.end()) return it->second;
  RecParams q{};
  q.H = d.H; q.U = c6.U; q.gs = c6.gs; q.rg = c6.rg; q.dirs = d.dirs; q.nwg = d.H / c6.U;
  size_t bytes = 0;
  g_rec6_probe = &bytes;
  try {
    launch6(fwd, d.mode, d.prec, c6.nth, q, dim3(1), 0, nullptr);
  } catch (...) {
    g_rec6_probe = nullptr;
    throw;
  }
  g_rec6_probe = nullptr;
  return memo[key] = bytes == 0;
}

// XCDs an XCD-pinned v6 recurrence of (d, N) occupies (bit x: XCD x), 0
// when it is not pinned: every (row group, direction) runs on one XCD, its
// H / U workgroups on kCusPerXcd (configs[1] / [4]: 32) or kCusPerXcd / 2
// (configs[2]: U = 32 at H = 512, four row groups x two directions = all
// eight XCDs, half of each XCD's CUs) of that XCD's CUs, and the whole chip's
// CUs must be usable (no CU partition).  KCTC_XCD6=0 / KCTC_XCD6F=0 switch it
// off; the 16-workgroup shapes pin too (configs[2]
// pinned: 990k -> 1.12M frames/s, forward 3.14 -> 2.42, backward 4.52 -> 3.53
// us/step, same box).
unsigned xcd_mask(const RnnDesc &d, int N, bool fwd) {
  const V6Cfg c6 = pick6(d, N, fwd);
  if (!c6 || d.dirs * c6.rg > 8) return 0;
  const int nwg = d.H / c6.U;
  if (nwg != kCusPerXcd && nwg != kCusPerXcd / 2) return 0;
  if (!env_int(fwd ? "KCTC_XCD6F" : "KCTC_XCD6", 1)) return 0;
  int dev = 0, cus = 0;
  KCTC_HIP_CHECK(hipGetDevice(&dev));
  KCTC_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  if (rnn_usable_cus() != cus || cus != 8 * kCusPerXcd) return 0;
  // backward: an exchange's kernels (comm stream) landing on a pinned XCD
  // would hold the recurrence's CUs there until the all-reduce ends, and a
  // stream CU mask cannot keep them off an XCD (scripts/cumask_probe.hip:
  // each mask bit selects one CU in every XCD): pinned only without an
  // exchange.  No exchange kernel runs during a forward pass (the previous
  // step's updates waited for every bucket), so the forward stays pinned.
  // With a residency-gated exchange (rnn_set_comm_gated) no exchange kernel
  // is in flight while a backward recurrence becomes resident, so it stays pinned.
  if (!fwd && rnn_comm_cus() > 0 && !rnn_comm_gated()) return 0;
  return (1u << (d.dirs * c6.rg)) - 1u;
}

// persistent blocks a streamed GEMM may run beside a recurrence of `rec_wgs`
// workgroups (rnn.h, CU budget); 0: too few to stream
int stream_block_budget(int rec_wgs, bool backward) {
  // the 16-CU margin keeps room for the exchange's kernels beyond maxCTAs;
  // a backward without an exchange (one rank) gives the streamed dx GEMM all
  // CUs the recurrence leaves (configs[1]: 128 blocks, 655.7k -> 670.7k frames/s)
  const int margin = backward && rnn_comm_cus() == 0 ? 0 : 16;
  const int left = rnn_usable_cus() - rec_wgs - (backward ? rnn_comm_cus() : 0) - margin;
  return left >= 8 ? left : 0;
}

// XCDs whose every CU an XCD-pinned recurrence holds: a streamed GEMM's
// blocks landing there leave at once (xcd_word / xcd_count), and the launch
// has 8 / (8 - pinned) times the blocks so that its budget stays.  0 when the
// recurrence is not pinned or its slots take half an XCD each (configs[2]:
// all eight XCDs, 16 of each XCD's CUs left to the stream: there its blocks
// stay, on the CUs the recurrence leaves).
int whole_pinned_xcds(const RecParams &p) {
  const int n = p.xpd && p.nwg == kCusPerXcd ? p.dirs * p.rg : 0;
  return n < 8 ? n : 0;
}

// Is the dx of layer l streamed off its v6 backward recurrence
// (launch_bwd_stream, given a dx buffer and an overlap stream)?  The
// forward's W^T prepack (RnnPrepack) asks the same question.
bool bwd_dx_stream_ok(const RnnDesc &d, int l, int T, int N) {
  const V6Cfg c6 = pick6(d, N, false);
  if (!c6 || d.dirs != 2 || !env_int("KCTC_BWD_STREAM", 1) || !rec6_scratch_free(d, N, false)) return false;
  // split-fp16 at N <= 16 by default (KCTC_STREAM_ALL: bf16 and N > 16 too)
  if (!((d.prec == kPrecX3 && N <= 16) || env_int("KCTC_STREAM_ALL", 0))) return false;
  const int G4 = d.nw() * d.H;
  if (!use_x3(G4) || G4 > 4096 || (d.prec != kPrecX3 && G4 % 64)) return false;
  if ((long)T * N * d.din(l) * 4 >= (1L << 31)) return false;
  return stream_block_budget(d.dirs * (d.H / c6.U) * c6.rg, true) > 0;
}

hipEvent_t fork_event(hipStream_t s) {
  static thread_local hipEvent_t ev = nullptr;
  if (!ev) KCTC_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  KCTC_HIP_CHECK(hipEventRecord(ev, s));
  return ev;
}
void join_stream(hipStream_t s, hipStream_t other) {
  static thread_local hipEvent_t ev = nullptr;
  if (!ev) KCTC_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  KCTC_HIP_CHECK(hipEventRecord(ev, other));
  KCTC_HIP_CHECK(hipStreamWaitEvent(s, ev, 0));
}

// Can `c` consume the exchange images of this component's last forward
// recurrence (v6, bidirectional) as its layer-0 projection input?
bool chain_ok(const RnnDesc &d, int ver, int T, int N, const RnnFwdChain *c) {
  if (!c || !c->d || !c->side || ver != 6 || d.dirs != 2 || !env_int("KCTC_FWD_STREAM", 1)) return false;
  if (!rec6_scratch_free(d, N, true)) return false;
  const RnnDesc &n = *c->d;
  // split-fp16 into split-fp16, or bf16 images into a bf16 projection
  if (n.D != d.dirs * d.H || !use_x3(n.D) || N > 64 || d.prec != n.prec) return false;
  // default: split-fp16 at N <= 16 only.  Row groups and bf16 run (and are
  // tested) under KCTC_STREAM_ALL=1, but are slower on the recipe shapes: at
  // N = 64 / T = 667 (configs[2]) and bf16 N = 32 (configs[4]) the GEMM on
  // the CUs left beside the 128-workgroup recurrence outlasts it (990k ->
  // 728k and 560k -> 389k frames/s measured), the 256-tile GEMM after it wins
  if ((N > 16 || d.prec == kPrecBf16) && !env_int("KCTC_STREAM_ALL", 0)) return false;
  // an XCD-pinned producer runs faster alone: beside the streamed projection
  // (HBM traffic on the other XCDs) its steps took 0.17-0.3 us longer, more
  // than the 256-tile GEMM after it costs (configs[1]: 555.9k vs 564.8k
  // frames/s same box); KCTC_FWD_STREAM_PINNED=1 streams anyway
  if (xcd_mask(d, N, true) && !env_int("KCTC_FWD_STREAM_PINNED", 0)) return false;
  // and only the IO-wave variant (U = 16, 512 threads) carries the copies
  // (launch6_u: U = 16 / 512 threads, not the stacked variant)
  if (xcd_mask(d, N, true) && !(pick6(d, N, true).U == 16 && pick6(d, N, true).nth == 512 &&
                                !(pick6(d, N, true).gs <= 8 && env_int("KCTC_STK_FWD", env_int("KCTC_STK", 1)))))
    return false;
  const V6Cfg c6 = pick6(d, N, true);
  if (!c6 || !stream_block_budget(d.dirs * (d.H / c6.U) * c6.rg, false)) return false;
  const long xs = 2L * (d.H / 32) * (d.prec == kPrecBf16 ? 1 : 2) * 16 * 32 * pick6(d, N, true).rg;  // halves per step image
  if ((long)T * xs * 2 >= (1L << 31)) return false;
  return c->ws_bytes >= rnn_workspace_bytes(n, T, N) &&
         c->res_bytes >= sizeof(float) * (size_t)rnn_reserve_layout(n, T, N).total;
}

// Layer-0 projection of the consumer, streamed off the producer's exchange images.
void launch_chain_proj(const RnnDesc &d, const RecParams &p, hipEvent_t fork, int T, int N, RnnFwdChain &c,
                       unsigned *err) {
  KCTC_HIP_CHECK(hipStreamWaitEvent(c.side, fork, 0));  // after the producer's flag reset
  beside_recurrence(c.side);
  const RnnDesc &n = *c.d;
  const bool bf = n.prec == kPrecBf16;
  const int NW = n.nw(), G = NW * n.H, Din = n.D, KB = Din / (bf ? 64 : 32);
  const long pl0 = n.lin_offset(0, 0, false), pls = n.pl_size(0);
  const float *wl = c.w + pl0;
  const PackLay pl = pack_layout(n, T, N);
  _Float16 *Bp = pk<_Float16>(c.workspace, n, T, N, pl.b);
  int *eB = bf ? nullptr : pk<int>(c.workspace, n, T, N, pl.eb);
  {
    ProfSpan ps(c.side, "x3_pack_chain");
    if (bf)
      bf16_pack_rows(c.side, wl, Din, G, Din, reinterpret_cast<__bf16 *>(Bp), n.dirs, pls, (long)G * KB * 64);
    else
      x3p_pack_rows(c.side, wl, Din, G, Din, Bp, eB, 0.f, n.dirs, pls, (long)G * KB * 64, (long)G);
  }
  const RnnReserveLayout lay = rnn_reserve_layout(n, T, N);
  X3PArgs x;
  x.bf16 = bf;
  x.M = T * N; x.N = G; x.KB = KB;
  x.A = reinterpret_cast<const _Float16 *>(p.xch); x.eA0 = bf ? 0 : 14;  // x3 images hold h 2^14
  x.B = Bp; x.eB = eB;
  x.C = static_cast<float *>(c.reserve) + lay.G; x.ldc = (long)n.dirs * G;
  x.bias = wl + (n.lin_offset(0, 0, true) - pl0);
  x.bias2 = n.mode == kGru ? nullptr : wl + (n.lin_offset(0, NW, true) - pl0);
  x.batch = n.dirs; x.sB = (long)G * KB * 64; x.seB = bf ? 0 : G; x.sC = G; x.sBias = pls;
  x.tile_counter = reinterpret_cast<int *>(static_cast<char *>(c.workspace) + flags_offset(n, T, N));
  // XCD-pinned producer: the sc1 copies of its epochs, no block on its XCDs
  x.stream_flags = p.flags + 1024 + (p.xpd ? 256 * kFlagStride : 0);  // pinned: agg_flag6 lines
  x.stream_nwg = p.xpd ? 1 : p.nwg; x.stream_T = T; x.stream_N = N;
  const int pinned = whole_pinned_xcds(p);
  if (pinned) { x.stream_xcd_word = p.flags + kXcdWord; x.stream_xcd_count = pinned; }
  x.stream_group_step = 2L * (d.H / 32) * (bf ? 1 : 2) * 16 * 32;  // rnn_fwd_rec6's XG
  x.stream_rg = p.rg; x.stream_gs = p.gs; x.stream_step = x.stream_group_step * p.rg; x.stream_err = err;
  // K split by producer direction: the work is ready from the first steps
  // (KCTC_STREAM_DIRSPLIT=0: whole-K tiles from the middle of the sequence outwards)
  if (env_int("KCTC_STREAM_DIRSPLIT", 1)) {
    x.stream_arrive = pk<int>(c.workspace, n, T, N, pl.fcnt);
    x.stream_part = pk<float>(c.workspace, n, T, N, pl.fpart);
  }
  // every producer workgroup needs a CU of its own (96 KB LDS); the GEMM's
  // persistent blocks (96 KB each) take the rest minus a margin (chain_ok
  // checked that at least 8 fit).  No gradient exchange runs during a
  // forward pass: the updates of the previous step waited for it.
  // (blocks landing on a pinned producer's XCDs exit at once: launch enough that the budget stays)
  const int nb = stream_block_budget(d.dirs * p.nwg * p.rg, false);
  x.max_blocks = pinned ? nb * 8 / (8 - pinned) : nb;
  {
    ProfSpan ps(c.side, "fwd_proj_stream");
    gemm_x3p(c.side, x);
  }
  c.done = true;
}

// Can `c`'s layer-0 projection stream off this component's y rows
// (launch_chain_rows)?  Split-fp16 into split-fp16, the 256-tile row stream.
bool chain_rows_ok(const RnnDesc &d, int ver, int T, int N, const RnnFwdChain *c) {
  if (!c || !c->d || !c->side || ver != 6 || d.dirs != 2 || d.prec == kPrecBf16 || !env_int("KCTC_FWD_STREAM", 1))
    return false;
  if (!rec6_scratch_free(d, N, true)) return false;
  const RnnDesc &n = *c->d;
  const long TN = (long)T * N;
  if (n.D != d.dirs * d.H || n.prec != d.prec || !use_x3(n.D) || d.H % 32 || d.H > 4096 || T < 2) return false;
  if (!x3p_bwd_stream_256((int)TN, n.dirs * n.nw() * n.H, d.H / 32, false)) return false;
  if (TN * n.dirs * n.nw() * n.H * 4 >= (1L << 31) || TN * (d.H / 32) * 128 >= (1L << 31)) return false;
  // at N <= 16 (configs[1]); larger batches run the 256-tile GEMM after the
  // recurrence (shorter recurrences, less time to hide the GEMM behind)
  if (N > 16 && !env_int("KCTC_STREAM_ALL", 0)) return false;
  const V6Cfg c6 = pick6(d, N, true);
  if (!c6 || !stream_block_budget(d.dirs * (d.H / c6.U) * c6.rg, false)) return false;
  return c->ws_bytes >= rnn_workspace_bytes(n, T, N) &&
         c->res_bytes >= sizeof(float) * (size_t)rnn_reserve_layout(n, T, N).total;
}

// The consumer's layer-0 projection G' = [y_fwd | y_bwd] W'^T + b' streamed
// off this forward recurrence's y rows (written through, p.ysc1): the
// direction-split row stream of gemm_x3p_bwd_stream with a forward producer --
// the K half of direction 0 of frame t is out at producer step t, direction
// 1's at step T - 1 - t, so each 256 x 256 tile of G' is two half-K jobs whose
// partials meet (plus the biases) in the second.  The K halves of W' are
// packed as rows of their own (per-half exponents).
void launch_chain_rows(const RnnDesc &d, const RecParams &p, hipEvent_t fork, int T, int N, RnnFwdChain &c,
                       unsigned *err) {
  KCTC_HIP_CHECK(hipStreamWaitEvent(c.side, fork, 0));  // after the producer's flag reset
  // not before every workgroup of the recurrence is resident: dispatched
  // first (another queue), 32 blocks per XCD would take every CU of an XCD
  // the recurrence is pinned to before its first workgroup got there (seen
  // once as a 3-s stream-wait timeout, error 0x2)
  beside_recurrence(c.side);
  const RnnDesc &n = *c.d;
  const int NW = n.nw(), G = NW * n.H, H = d.H, KBh = H / 32, Din = n.D;
  const long TN = (long)T * N;
  const long pl0 = n.lin_offset(0, 0, false), pls = n.pl_size(0);
  const float *wl = c.w + pl0;
  const PackLay pl = pack_layout(n, T, N);
  _Float16 *Bp = pk<_Float16>(c.workspace, n, T, N, pl.b);
  int *eB = pk<int>(c.workspace, n, T, N, pl.eb);
  const long sB = (long)n.dirs * G * KBh * 64;
  {
    ProfSpan ps(c.side, "x3_pack_chain");
    for (int h = 0; h < 2; h++)  // K half h of the rows of both consumer directions
      x3p_pack_rows(c.side, wl + h * H, Din, G, H, Bp + h * sB, eB + h * n.dirs * G, 0.f, n.dirs, pls,
                    (long)G * KBh * 64, G);
  }
  const RnnReserveLayout lay = rnn_reserve_layout(n, T, N);
  X3PBwdStream a;
  a.forward = true;
  a.M = (int)TN; a.N = n.dirs * G; a.KB = KBh;
  a.E = p.y; a.lde = 2L * H; a.edoff = H;
  a.Ap = pk<_Float16>(c.workspace, n, T, N, pl.a); a.eA = pk<int>(c.workspace, n, T, N, pl.ea);
  a.B = Bp; a.eB = eB; a.sB = sB; a.seB = n.dirs * G;
  a.C = static_cast<float *>(c.reserve) + lay.G; a.ldc = (long)n.dirs * G;
  a.bias = wl + (n.lin_offset(0, 0, true) - pl0);
  a.bias2 = n.mode == kGru ? nullptr : wl + (n.lin_offset(0, NW, true) - pl0);
  a.bias_cols = G; a.sbias = pls;
  a.part = pk<float>(c.workspace, n, T, N, pl.fpart);
  a.part2 = pk<float>(c.workspace, n, T, N, pl.part2);
  a.cnt = pk<int>(c.workspace, n, T, N, pl.cnt);
  a.flags = p.flags + 1024 + (p.xpd ? 256 * kFlagStride : 0);  // pinned: agg_flag6 lines
  a.nwg = p.xpd ? 1 : p.nwg; a.T = T; a.Nf = N; a.err = err; a.rg = p.rg;
  const int pinned = whole_pinned_xcds(p);
  if (pinned) { a.xcd_word = p.flags + kXcdWord; a.xcd_count = pinned; }
  // 128: every CU the recurrence leaves (configs[1]: 96 -> 128 blocks 720k -> 751k frames/s)
  const int nb = std::min(128, stream_block_budget(d.dirs * p.nwg * p.rg, false));
  a.blocks = pinned ? nb * 8 / (8 - pinned) : nb;
  {
    ProfSpan ps(c.side, "fwd_proj_rows");
    gemm_x3p_bwd_stream(c.side, a);
  }
  c.done = true;
}

}  // namespace

void rnn_set_cu_budget(int cus, int comm) {
  g_usable_cus = std::max(0, cus);
  g_comm_cus = std::max(0, comm);
}
int rnn_usable_cus() {
  static int dev_cus[64] = {0};
  int dev = 0;
  KCTC_HIP_CHECK(hipGetDevice(&dev));
  int &c = dev_cus[dev & 63];
  if (!c) KCTC_HIP_CHECK(hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev));
  return g_usable_cus > 0 ? std::min(g_usable_cus, c) : c;
}
int rnn_comm_cus() { return g_comm_cus; }

// ---- residency gate of the gradient exchange (rnn.h) ----
namespace {
struct RegWord {
  unsigned *word = nullptr;          // [1]: gate timeouts, [2]: pinned XCDs, [4..5]: registrations (64-bit: never wraps),
                                     // [6]: exchange gate blocks gone (rnn_comm_gate)
  unsigned long long expected = 0;   // host: registrations once every enqueued launch is resident
};
RegWord g_reg[64];
int g_comm_gated[64] = {0};  // per device: live gated exchanges (at most one, GatedExchange)
int current_device() {
  int dev = 0;
  KCTC_HIP_CHECK(hipGetDevice(&dev));
  return dev & 63;
}
RegWord &reg_of_device() {
  int dev = 0;
  KCTC_HIP_CHECK(hipGetDevice(&dev));
  RegWord &r = g_reg[dev & 63];
  if (!r.word) {
    KCTC_HIP_CHECK(hipMalloc(&r.word, 256));
    KCTC_HIP_CHECK(hipMemset(r.word, 0, 256));
  }
  return r;
}
}  // namespace

// The gates poll the word (10 s at most, then they give up and set bit 0 of
// the device word's [1]).  hipStreamWaitValue is no alternative: ROCclr runs
// it as a one-thread kernel too (__amd_rocclr_streamOpsWait), without a
// timeout -- under rocprofv3's counter collection, which serialises
// dispatches, a gate dispatched before its recurrence then never returns.
// A gate is kGateBlocks one-wave blocks, one per XCD (round-robin dispatch).
// A wave of it holds a CU, and a recurrence workgroup that needs a CU's whole
// register file (configs[4]'s bf16 GRU backward: 256 VGPRs x 2 waves per
// SIMD) cannot be placed beside it: a gate on one of the 32 CUs of an XCD the
// recurrence is pinned to kept that XCD's last workgroup out until the gate
// timed out (error 0x10003 at configs[4] with KCTC_STREAM_ALL=1).  So a block
// leaves as soon as the recurrence has a workgroup on its own XCD (xw: the
// XCD bits its workgroups OR in first thing), unless it is the last block
// still waiting (leave counts the ones gone): the blocks on XCDs the
// recurrence does not use do the waiting.  (A full-register recurrence on all
// eight XCDs would keep the last block's CU; no recipe shape is one -- with
// every CU taken nothing streams beside it either -- and the gate's timeout
// would flag it.)
constexpr int kGateBlocks = 8;
template <typename W>
__global__ __launch_bounds__(64) void gate_kernel(const W *word, W target, unsigned *gerr, const unsigned *xw,
                                                  unsigned *leave) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned me = 1u << xcc_id();
  bool late = false;
  while (true) {
    const W v = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__builtin_amdgcn_readfirstlane((int)(v >= target))) break;
    if (xw && __builtin_amdgcn_readfirstlane((int)(__hip_atomic_load(xw, __ATOMIC_RELAXED,
                                                                     __HIP_MEMORY_SCOPE_AGENT) & me))) {
      unsigned gone = 0;
      if (threadIdx.x == 0) gone = atomicAdd(leave, 1u);
      if (__builtin_amdgcn_readfirstlane((int)gone) < kGateBlocks - 1) return;
      xw = nullptr;  // the last one: it stays
    }
    late = __builtin_amdgcn_s_memrealtime() - t0 > 1000000000ull;  // 100 MHz clock
    if (late) break;
    __builtin_amdgcn_s_sleep(8);
  }
  if (late && threadIdx.x == 0) atomicOr(gerr, 1u);
}

unsigned long long rnn_bwd_registrations() { return reg_of_device().expected; }
void rnn_resident_gate(hipStream_t s, const unsigned *flags, unsigned target) {
  hipLaunchKernelGGL(gate_kernel<unsigned>, dim3(kGateBlocks), dim3(64), 0, s, flags + kResWord, target,
                     reg_of_device().word + 1, flags + kXcdWord, const_cast<unsigned *>(flags) + kGateWord);
  KCTC_HIP_CHECK(hipGetLastError());
}
const unsigned *rnn_pinned_xcds() { return reg_of_device().word + 2; }

void rnn_comm_gate(hipStream_t s, unsigned long long target) {
  RegWord &r = reg_of_device();
  // XCDs of the pinned backward recurrences (word [2], never cleared); the
  // blocks gone counted in word [6], zeroed per gate on its own stream
  KCTC_HIP_CHECK(hipMemsetAsync(r.word + 6, 0, sizeof(unsigned), s));
  hipLaunchKernelGGL(gate_kernel<unsigned long long>, dim3(kGateBlocks), dim3(64), 0, s,
                     reinterpret_cast<const unsigned long long *>(r.word + 4), target, r.word + 1, r.word + 2,
                     r.word + 6);
  KCTC_HIP_CHECK(hipGetLastError());
}
void rnn_set_comm_gated(bool on) {
  int &c = g_comm_gated[current_device()];
  c = on ? c + 1 : std::max(0, c - 1);
}
bool rnn_comm_gated() { return g_comm_gated[current_device()] > 0; }

bool rnn_packed_output(const RnnDesc &d, int T, int N, void *reserve, const void **rows, const void **cols) {
  *rows = *cols = nullptr;
  if (!bf16_io(d) || !reserve) return false;
  const RnnReserveLayout lay = rnn_reserve_layout(d, T, N);
  float *res = static_cast<float *>(reserve);
  *rows = res + lay.pkyr;
  *cols = res + lay.pkyc;
  return true;
}

namespace {
void pack_dx_weights(const RnnDesc &d, int l, const float *w, void *workspace, int T, int N, hipStream_t st);
}  // namespace

int rnn_forward_training(const RnnDesc &d, hipStream_t s, int T, int N, const float *x,
                         const float *w, float *y, void *workspace, size_t ws_bytes,
                         void *reserve, size_t res_bytes, unsigned *err, RnnFwdChain *chain,
                         bool input_projected, const void *in_rows, RnnPrepack *pre) {
  RecScope rec_scope;  // the side launches' residency gates (beside_recurrence)
  if (chain) chain->done = false;
  if (pre) pre->done = pre->wdone = false;
  if (T <= 0 || N <= 0 || N > 16 * kMaxRT || d.H % 16) return KRNN_NOT_SUPPORTED;
  const RnnReserveLayout lay = rnn_reserve_layout(d, T, N);
  if (res_bytes < sizeof(float) * (size_t)lay.total) return KRNN_BAD_PARAM;
  if (ws_bytes < rnn_workspace_bytes(d, T, N)) return KRNN_BAD_PARAM;
  const V6Cfg c6 = pick6(d, N, true);
  const int U6 = c6.U;
  const int U4 = U6 ? 0 : pick_fwd_u4(d, N);
  const int ver = U6 ? 6 : U4 ? 4 : 3;
  const int U = U6 ? U6 : U4 ? U4 : pick_fwd_u(d, N);
  if (d.prec == kPrecBf16 && ver != 6) return KRNN_NOT_SUPPORTED;  // bf16 exists on v6 only
  if (!U) return KRNN_NOT_SUPPORTED;
  const int NW = d.nw(), H = d.H, dirs = d.dirs;
  const long TN = (long)T * N;
  float *res = static_cast<float *>(reserve);
  const float *in = x;
  for (int l = 0; l < d.layers; l++) {
    float *R0 = res + lay.per_layer * l;
    float *out = (l == d.layers - 1) ? y : R0 + lay.out;
    const int Din = d.din(l);
    const long pl0 = d.lin_offset(l * dirs, 0, false);
    const float *wl = w + pl0;
    const long pls = d.pl_size(l);
    const long bW = d.lin_offset(l * dirs, 0, true) - pl0;
    const long bR = d.lin_offset(l * dirs, NW, true) - pl0;
    const long roff = d.lin_offset(l * dirs, NW, false) - pl0;
    if (ver == 3) KCTC_HIP_CHECK(hipMemsetAsync(out, 0xFF, sizeof(float) * TN * dirs * H, s));
    GemmArgs g;
    g.transA = false; g.transB = true;
    g.M = (int)TN; g.N = NW * H; g.K = Din;
    const bool skip_proj = l == 0 && input_projected;  // streamed by the previous component
    g.A = in; g.lda = Din;
    g.B = wl; g.ldb = Din;
    g.C = R0 + lay.G; g.ldc = (long)dirs * NW * H;
    g.bias = wl + bW;
    g.bias2 = (d.mode == kGru) ? nullptr : wl + bR;
    g.batch = dirs; g.strideA = 0; g.strideB = pls; g.strideC = (long)NW * H; g.strideBias = pls;
    if (skip_proj) {
    } else if (d.prec == kPrecBf16 && use_x3(Din, 32)) {
      // bf16 gate GEMM: input rows and W rows packed as bf16, fp32 accumulation
      const PackLay pl = pack_layout(d, T, N);
      // the input rows come packed from the previous component's forward (in_rows)
      const bool rows_in = l == 0 && in_rows && Din % 64 == 0;
      __bf16 *Ap = rows_in ? static_cast<__bf16 *>(const_cast<void *>(in_rows)) : pk<__bf16>(workspace, d, T, N, pl.a);
      __bf16 *Bp = pk<__bf16>(workspace, d, T, N, pl.b);
      const int KB = (Din + 63) / 64;
      {
        ProfSpan ps(s, "x3_pack");
        if (!rows_in) bf16_pack_rows(s, in, Din, (int)TN, Din, Ap);
        bf16_pack_rows(s, wl, Din, NW * H, Din, Bp, dirs, pls, (long)NW * H * KB * 64);
      }
      X3PArgs x;
      x.bf16 = true;
      x.M = (int)TN; x.N = NW * H; x.KB = KB;
      x.A = reinterpret_cast<const _Float16 *>(Ap); x.B = reinterpret_cast<const _Float16 *>(Bp);
      x.C = g.C; x.ldc = g.ldc; x.bias = g.bias; x.bias2 = g.bias2;
      x.batch = dirs; x.sA = 0; x.sB = (long)NW * H * KB * 64;
      x.sC = g.strideC; x.sBias = g.strideBias;
      ProfSpan ps(s, "gemm_fwd_proj");
      gemm_x3p(s, x);
    } else if (use_x3(Din, 32)) {
      // input rows (a lower stacked layer's output is bounded; the component
      // input and RELU outputs get per-row exponents) and W rows, packed
      const PackLay pl = pack_layout(d, T, N);
      _Float16 *Ap = pk<_Float16>(workspace, d, T, N, pl.a), *Bp = pk<_Float16>(workspace, d, T, N, pl.b);
      int *eA = pk<int>(workspace, d, T, N, pl.ea), *eB = pk<int>(workspace, d, T, N, pl.eb);
      const int KB = (Din + 31) / 32;
      {
        ProfSpan ps(s, "x3_pack");
        x3p_pack_rows(s, in, Din, (int)TN, Din, Ap, eA, (l > 0 && bounded_out(d)) ? 1.f : 0.f);
        x3p_pack_rows(s, wl, Din, NW * H, Din, Bp, eB, 0.f, dirs, pls, (long)NW * H * KB * 64, (long)NW * H);
      }
      X3PArgs x;
      x.M = (int)TN; x.N = NW * H; x.KB = KB;
      x.A = Ap; x.B = Bp; x.eA = eA; x.eB = eB;
      x.C = g.C; x.ldc = g.ldc; x.bias = g.bias; x.bias2 = g.bias2;
      x.batch = dirs; x.sA = 0; x.seA = 0; x.sB = (long)NW * H * KB * 64; x.seB = (long)NW * H;
      x.sC = g.strideC; x.sBias = g.strideBias;
      ProfSpan ps(s, "gemm_fwd_proj");
      gemm_x3p(s, x);
    } else {
      ProfSpan ps(s, "gemm_fwd_proj");
      gemm_f32(s, g);
    }
    RecParams p{};
    p.T = T; p.N = N; p.H = H; p.dirs = dirs; p.U = U; p.nwg = H / U;
    p.ncol = (NW * U + 15) / 16 * 16; p.Npad = (N + 15) / 16 * 16;
    p.w = wl; p.pl_stride = pls; p.r_off = roff; p.bR_off = bR;
    p.G = R0 + lay.G; p.y = out; p.aux = R0 + lay.aux; p.err = err;
    p.sync = ver == 4 ? kSyncFlag : kSyncData;
    p.allow_local = 0;
    p.flags = reinterpret_cast<unsigned *>(static_cast<char *>(workspace) + flags_offset(d, T, N));
    KCTC_HIP_CHECK(hipMemsetAsync(p.flags, 0, kFlagBytes, s));
    const size_t lds = ver == 6 ? fwd6_lds_bytes(d, c6) : fwd_lds_bytes(d, N, U);
    p.xpd = ver == 4 ? v4_xpd(d, U) : 1;
    p.rg = ver == 6 ? c6.rg : 1;
    p.gs = ver == 6 ? c6.gs : 16;
    p.xch = reinterpret_cast<float *>(static_cast<char *>(workspace) + xch_offset(d, T, N));
    p.poll_sleep = 1;
    p.gla = 3;  // G rows fetched 3 steps ahead (IO waves)
    if (ver == 6 && bf16_io(d)) {  // the output also as packed bf16 rows and columns
      p.yr = reinterpret_cast<__bf16 *>(R0 + lay.pkyr);
      p.yc = reinterpret_cast<__bf16 *>(R0 + lay.pkyc);
      p.kbt64 = lay.kbt64;
      if (lay.kbt64 > TN)
        KCTC_HIP_CHECK(hipMemset2DAsync(p.yc + TN, sizeof(__bf16) * lay.kbt64, 0, sizeof(__bf16) * (lay.kbt64 - TN),
                                        (size_t)dirs * H, s));
    }
    const bool chained = l == d.layers - 1 && chain_ok(d, ver, T, N, chain);
    const bool rowchain = !chained && l == d.layers - 1 && chain_rows_ok(d, ver, T, N, chain);
    if (ver == 6) {
      // XCD-pinned forward (xcd_mask): each (row group, direction) on one XCD,
      // the h hand-off in its L2 through a ring of two step images; a
      // streamed projection gets sc1 copies of the step images and flags
      p.xpd = xcd_mask(d, N, true) ? 1 : 0;
      p.ring = p.xpd ? 2 : 0;
      p.fcopy = p.xpd && chained;
      p.ysc1 = rowchain ? 1 : 0;
      p.allow_local = p.xpd ? 1 : 0;
      // self-tagged hand-off (the kernel takes it for split-fp16 without IO
      // waves or a write-through copy): the ring's two images start at tag 1
      p.dtag = d.prec != kPrecBf16 && p.ring == 2 && !p.fcopy && T >= 2;
      if (p.dtag) {  // rnn_fwd_rec6's ring: after T step images of XS = 64 H rg halves (2 dirs, hi / lo, 16 rows)
        const size_t xs = sizeof(_Float16) * 64 * (size_t)d.H * p.rg;
        KCTC_HIP_CHECK(hipMemsetAsync(reinterpret_cast<char *>(p.xch) + xs * T, 0x01, 2 * xs, s));
      }
    }
    const dim3 grid(ver == 4 ? 8 * ceil_div(p.nwg, p.xpd) : ver == 6 && p.xpd ? 8 * p.nwg : dirs * p.nwg * p.rg);
    RecTrace tr;
    if (tr.arm("fwd", grid.x)) p.trace = tr.dev;
    // W^T of the backward's streamed dx GEMM, packed beside this recurrence
    // (rnn_backward_data's `streamed` shapes; one-layer descriptors)
    const bool prepack = pre && pre->dx && pre->stream && pre->ev && ver == 6 && d.layers == 1 &&
                         bwd_dx_stream_ok(d, 0, T, N);
    const bool prepack_w = pre && pre->stream && pre->wev && pre->wgrad && pre->in_bound > 0.f && ver == 6 &&
                           d.layers == 1 && d.prec != kPrecBf16 && T > 1 && bounded_out(d) && use_x3((int)TN) &&
                           rec6_scratch_free(d, N, true);
    const hipEvent_t fork = (chained || prepack || prepack_w || rowchain) ? fork_event(s) : nullptr;
    {
      ProfSpan ps(s, "rnn_fwd_rec");
      if (ver == 6) launch6(true, d.mode, d.prec, c6.nth, p, grid, lds, s);
      else launch_rec(true, d.mode, p, grid, lds, s, ver);
    }
    KCTC_HIP_CHECK(hipGetLastError());
    if (ver == 6) rec_scope.enqueued(p);
    else rec_scope.none();
    if (prepack) {  // beside the recurrence, once it is resident
      KCTC_HIP_CHECK(hipStreamWaitEvent(pre->stream, fork, 0));
      beside_recurrence(pre->stream);
      pack_dx_weights(d, 0, w, workspace, T, N, pre->stream);
      KCTC_HIP_CHECK(hipEventRecord(pre->ev, pre->stream));
      pre->done = true;
    }
    if (prepack_w) {  // x^T beside the recurrence, y^T after it, off its XCDs (rnn_backward_weights' packs)
      hipStream_t ss = pre->stream;
      if (!prepack) KCTC_HIP_CHECK(hipStreamWaitEvent(ss, fork, 0));
      beside_recurrence(ss);
      const PackLay pl = pack_layout(d, T, N);
      const int Din = d.din(0);
      int *pc = pk<int>(workspace, d, T, N, pl.pcnt);  // item counters
      KCTC_HIP_CHECK(hipMemsetAsync(pc, 0, sizeof(int) * 3, ss));
      const unsigned *av = rnn_pinned_xcds();
      const int nx = std::max(1, rnn_usable_cus() / kCusPerXcd);
      ProfSpan ps(ss, "x3_pack_w_fwd");
      x3p_pack_cols(ss, in, Din, (int)TN, Din, 0, pk<_Float16>(workspace, d, T, N, pl.xt),
                    pk<int>(workspace, d, T, N, pl.ext), nullptr, pre->in_bound, 1, 0, 0, 0, 0, av, nx, pc);
    }
    if (chained) {
      launch_chain_proj(d, p, fork, T, N, *chain, err);
      join_stream(s, chain->side);
    }
    if (rowchain) {
      launch_chain_rows(d, p, fork, T, N, *chain, err);
      join_stream(s, chain->side);
    }
    if (prepack_w) {  // y^T after the recurrence (and after the joins: s does not wait for it)
      hipStream_t ss = pre->stream;
      KCTC_HIP_CHECK(hipStreamWaitEvent(ss, fork_event(s), 0));
      const PackLay pl = pack_layout(d, T, N);
      const long KBt = (TN + 31) / 32;
      int *pc = pk<int>(workspace, d, T, N, pl.pcnt);
      const unsigned *av = rnn_pinned_xcds();
      const int nx = std::max(1, rnn_usable_cus() / kCusPerXcd);
      const long ldy = (long)dirs * H;
      {
        ProfSpan ps(ss, "x3_pack_w_fwd");
        for (int dir = 0; dir < dirs; dir++)
          x3p_pack_cols(ss, out + (long)dir * H, ldy, (int)TN, H, dir == 0 ? N : -N,
                        pk<_Float16>(workspace, d, T, N, pl.yt) + (long)dir * H * KBt * 64,
                        pk<int>(workspace, d, T, N, pl.eyt) + dir * H, nullptr, 1.f, 1, 0, 0, 0, 0, av, nx,
                        pc + 1 + dir);
      }
      KCTC_HIP_CHECK(hipEventRecord(pre->wev, ss));
      pre->wdone = true;
    }
    tr.dump("fwd", s, grid.x, p.nwg, T, dirs, ver, ver == 6 ? (p.xpd ? 1 : 0) : p.xpd);
    in = out;
  }
  return KRNN_OK;
}

namespace {
// dx of stacked layer l on `ov`, streamed off the backward recurrence about
// to be launched on `s` (gemm_x3p_bwd_stream): W_d^T packed first, then one
// persistent launch that packs dGates rows as the recurrence flags them.
// W^T of layer l's dx GEMM (B operand of the streamed GEMM) into the
// workspace slot pl.wt (per-column exponents pl.ewt, absmax scratch pl.cmw)
void pack_dx_weights(const RnnDesc &d, int l, const float *w, void *workspace, int T, int N, hipStream_t st) {
  const bool bf = d.prec == kPrecBf16;
  const int G4 = d.nw() * d.H, KB = G4 / (bf ? 64 : 32), Din = d.din(l);
  const long pl0 = d.lin_offset(l * d.dirs, 0, false), pls = d.pl_size(l);
  const float *wl = w + pl0;
  const PackLay pl = pack_layout(d, T, N);
  _Float16 *Bp = pk<_Float16>(workspace, d, T, N, pl.wt);
  int *eB = pk<int>(workspace, d, T, N, pl.ewt);
  unsigned *cm = pk<unsigned>(workspace, d, T, N, pl.cmw);
  ProfSpan ps(st, "x3_pack_bwd_stream");
  for (int dir = 0; dir < 2; dir++) {
    if (bf) {
      bf16_pack_cols(st, wl + dir * pls, Din, G4, Din, 0, reinterpret_cast<__bf16 *>(Bp) + (long)dir * Din * KB * 64);
      continue;
    }
    absmax_f32(st, wl + dir * pls, Din, G4, Din, nullptr, cm + dir * Din);
    x3p_pack_cols(st, wl + dir * pls, Din, G4, Din, 0, Bp + (long)dir * Din * KB * 64, eB + dir * Din, cm + dir * Din,
                  0.f);
  }
}

void launch_bwd_stream(const RnnDesc &d, const RecParams &p, int l, const float *w, float *dxl, void *workspace,
                       int T, int N, hipStream_t ov, hipEvent_t fork, unsigned *err, const RnnPrepack *pre) {
  KCTC_HIP_CHECK(hipStreamWaitEvent(ov, fork, 0));  // after the flag reset, not after the recurrence
  // not before every workgroup of the recurrence is resident: its blocks
  // wait (on_pinned_xcd) for the pinned recurrence's XCDs to register, and a
  // block parked on one of those XCDs' CUs before the recurrence's last
  // workgroup got there would keep it out (with W^T packed by the forward
  // the GEMM starts together with the recurrence)
  beside_recurrence(ov);
  const bool bf = d.prec == kPrecBf16;
  const int NW = d.nw(), H = d.H, G4 = NW * H, KB = G4 / (bf ? 64 : 32), Din = d.din(l);
  const long TN = (long)T * N;
  const PackLay pl = pack_layout(d, T, N);
  _Float16 *Ap = pk<_Float16>(workspace, d, T, N, pl.a), *Bp = pk<_Float16>(workspace, d, T, N, pl.wt);
  int *eA = pk<int>(workspace, d, T, N, pl.ea), *eB = pk<int>(workspace, d, T, N, pl.ewt);
  // packed by the forward on its side stream (RnnPrepack), else here
  if (pre && pre->done) KCTC_HIP_CHECK(hipStreamWaitEvent(ov, pre->ev, 0));
  else pack_dx_weights(d, l, w, workspace, T, N, ov);
  X3PBwdStream a;
  a.bf16 = bf;
  a.M = (int)TN; a.N = Din; a.KB = KB;
  a.E = p.DX; a.lde = 2L * G4; a.edoff = G4;
  a.Ap = Ap; a.eA = eA;
  a.B = Bp; a.eB = bf ? nullptr : eB; a.sB = (long)Din * KB * 64; a.seB = Din;
  a.C = dxl; a.ldc = Din;
  a.part = pk<float>(workspace, d, T, N, pl.part);
  a.part2 = pk<float>(workspace, d, T, N, pl.part2);
  a.cnt = pk<int>(workspace, d, T, N, pl.cnt);
  // XCD-pinned recurrence: its epochs' sc1 copies (the L2 flags are not
  // visible here), and no block on the recurrence's XCDs
  a.flags = p.flags + 1024 + (p.xpd ? 256 * kFlagStride : 0);  // pinned: agg_flag6 lines
  a.nwg = p.xpd ? 1 : p.nwg; a.T = T; a.Nf = N; a.err = err; a.rg = p.rg;
  const int pinned = whole_pinned_xcds(p);
  if (pinned) { a.xcd_word = p.flags + kXcdWord; a.xcd_count = pinned; }
  // 128 measured best at configs[1] since the self-tagged recurrences (96
  // before: 655.7k -> 670.7k frames/s); never more than the CU budget leaves
  // beside the recurrence and the exchange's kernels (rnn.h).  Blocks landing
  // on the pinned XCDs exit at once: launch enough that ~128 stay
  // 256-tile launch: 48 blocks keep up with the recurrence and leave the
  // other CUs beside it to the weight GEMMs (rnn_backward_weights beside)
  const bool t256 = x3p_bwd_stream_256(a.M, a.N, a.KB, bf);
  const int nb = std::min(t256 ? 64 : 128,
                          stream_block_budget(d.dirs * p.nwg * p.rg, true));
  a.blocks = pinned ? nb * 8 / (8 - pinned) : nb;
  ProfSpan ps(ov, "bwd_data_stream");
  gemm_x3p_bwd_stream(ov, a);
}
}  // namespace

// ---------------------------------------------------------------------------
// streamed weight gradients of the bottom component (rnn.h RnnWgradStream)
// ---------------------------------------------------------------------------
namespace {
// One wave: returns once every v6 flag line (stride kFlagStride words) holds
// >= epoch, the recurrence reported an error, or after 3 s (then err bit 3).
// Every exit decision is wave-uniform; the error store follows the loop.
__global__ __launch_bounds__(64) void rec_gate_kernel(const unsigned *flags, int nlines, unsigned epoch,
                                                      unsigned *err) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int spins = 0;
  bool late = false;
  while (true) {
    bool ok = true;
    for (int i = threadIdx.x; i < nlines; i += 64)
      ok &= __hip_atomic_load(flags + (long)i * kFlagStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= epoch;
    if (__all(ok)) break;
    if ((++spins & 255) == 0) {
      const unsigned e = __builtin_amdgcn_readfirstlane(__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      if (e) break;
      late = __builtin_amdgcn_s_memrealtime() - t0 > 300000000ull;
      if (late) break;
    }
    __builtin_amdgcn_s_sleep(16);
  }
  if (late && threadIdx.x == 0) atomicOr(err, 8u);
}

// dW_dir += DX_dir^T x and dR_dir += DX_dir^T h_prev over the frames [ta, tb)
// of direction dir (layer 0 of a one-layer component, split-fp16, LSTM: E == DX)
void wgrad_frames(const RnnDesc &d, hipStream_t s, int T, int N, const float *x, const float *y, void *workspace,
                  float *dw, void *reserve, int max_blocks, float in_bound, int dir, int ta, int tb) {
  if (tb <= ta) return;
  const RnnReserveLayout lay = rnn_reserve_layout(d, T, N);
  const int NW = d.nw(), H = d.H, dirs = d.dirs, G4 = NW * H, Din = d.din(0);
  const long ldg = (long)dirs * G4, ldy = (long)dirs * H;
  const int R = (tb - ta) * N, KB = (R + 31) / 32;
  const float *DX = static_cast<const float *>(reserve) + lay.E;
  const PackLay pl = pack_layout(d, T, N);
  _Float16 *DXt = pk<_Float16>(workspace, d, T, N, pl.a), *Xt = pk<_Float16>(workspace, d, T, N, pl.b);
  _Float16 *Yt = pk<_Float16>(workspace, d, T, N, pl.c);
  int *eDX = pk<int>(workspace, d, T, N, pl.ea), *eX = pk<int>(workspace, d, T, N, pl.eb);
  int *eY = pk<int>(workspace, d, T, N, pl.ec);
  unsigned *cm = pk<unsigned>(workspace, d, T, N, pl.cm);
  unsigned *fl = reinterpret_cast<unsigned *>(static_cast<char *>(workspace) + flags_offset(d, T, N));
  float *ws = static_cast<float *>(workspace);
  const long ws_floats = drec_split_floats(d, T, N);
  {
    ProfSpan ps(s, "x3_pack_w");
    const float *src = DX + (long)ta * N * ldg + (long)dir * G4;
    absmax_f32(s, src, ldg, R, G4, nullptr, cm);
    x3p_pack_cols(s, src, ldg, R, G4, 0, DXt, eDX, cm, 0.f);
    const float *xs = x + (long)ta * N * Din;
    if (!(in_bound > 0.f)) absmax_f32(s, xs, Din, R, Din, nullptr, cm + G4);
    x3p_pack_cols(s, xs, Din, R, Din, 0, Xt, eX, cm + G4, in_bound > 0.f ? in_bound : 0.f);
    // h_prev: direction 0 pairs frame t with y(t - 1), direction 1 with y(t + 1);
    // frames outside the sequence contribute zero (pack_cols zero-fills k - shift outside [0, R))
    const float *yd = y + (long)dir * H;
    if (dir == 0) {
      if (ta == 0) x3p_pack_cols(s, yd, ldy, R, H, N, Yt, eY, nullptr, 1.f);
      else x3p_pack_cols(s, yd + (long)(ta - 1) * N * ldy, ldy, R, H, 0, Yt, eY, nullptr, 1.f);
    } else {
      if (tb == T) x3p_pack_cols(s, yd + (long)ta * N * ldy, ldy, R, H, -N, Yt, eY, nullptr, 1.f);
      else x3p_pack_cols(s, yd + (long)(ta + 1) * N * ldy, ldy, R, H, 0, Yt, eY, nullptr, 1.f);
    }
  }
  auto split_for = [&](int n) {
    int sp = x3p_pick_split(G4, n, KB, 1);
    while (sp > 1 && (long)sp * G4 * n > ws_floats) sp--;
    return sp;
  };
  const long pl0 = d.lin_offset(dir, 0, false);
  {
    X3PArgs a;
    a.M = G4; a.N = Din; a.KB = KB;
    a.A = DXt; a.eA = eDX; a.B = Xt; a.eB = eX;
    a.C = dw + pl0; a.ldc = Din; a.beta = 1.f; a.batch = 1;
    a.split_k = split_for(Din); a.ws = ws;
    a.max_blocks = max_blocks;
    if (max_blocks > 0) a.tile_counter = reinterpret_cast<int *>(fl + 1008);
    ProfSpan ps(s, "gemm_bwd_w");
    gemm_x3p(s, a);
  }
  {
    X3PArgs a;
    a.M = G4; a.N = H; a.KB = KB;
    a.A = DXt; a.eA = eDX; a.B = Yt; a.eB = eY;
    a.C = dw + d.lin_offset(dir, NW, false); a.ldc = H; a.beta = 1.f; a.batch = 1;
    a.split_k = split_for(H); a.ws = ws;
    a.max_blocks = max_blocks;
    if (max_blocks > 0) a.tile_counter = reinterpret_cast<int *>(fl + 1009);
    ProfSpan ps(s, "gemm_bwd_r");
    gemm_x3p(s, a);
  }
}

// dbW += sum dGx, dbR += sum dGh of layer l from the recurrence's per-group partials
void wgrad_bias(const RnnDesc &d, hipStream_t s, int T, int N, float *dw, void *reserve, int l) {
  const RnnReserveLayout lay = rnn_reserve_layout(d, T, N);
  const int NW = d.nw(), H = d.H, dirs = d.dirs, G4 = NW * H;
  const float *R0 = static_cast<const float *>(reserve) + lay.per_layer * l;
  const long pl0 = d.lin_offset(l * dirs, 0, false), pls = d.pl_size(l);
  float *dwl = dw + pl0;
  const long bW = d.lin_offset(l * dirs, 0, true) - pl0;
  const long bR = d.lin_offset(l * dirs, NW, true) - pl0;
  // (v6: one partial per row group, [group][dir][2][G], added in group order)
  const V6Cfg c6b = pick6(d, N, false);
  const int rg = c6b ? c6b.rg : 1;
  for (int gi = 0; gi < rg; gi++)
    for (int dir = 0; dir < dirs; dir++) {
      const float *part = R0 + lay.bias + ((long)gi * dirs + dir) * 2 * G4;
      clip_sgd_update(s, dwl + dir * pls + bW, part, G4, 1.f, 0.f);
      clip_sgd_update(s, dwl + dir * pls + bR, part + G4, G4, 1.f, 0.f);
    }
}
}  // namespace

// Off by default (KCTC_WGRAD_STREAM=1 turns it on): measured on configs[1]
// 470.4k -> 467.0k (2 chunks), 466.1k (4), 454.5k (8) frames/s: the chunk
// GEMMs beside the backward recurrence slow it (33.0 -> 33.3-33.5 ms/step)
// and the per-chunk transposes add packing, more than the 1 ms tail saved.
bool rnn_wgrad_stream_ok(const RnnDesc &d, int T, int N) {
  if (!env_int("KCTC_WGRAD_STREAM", 0) || d.layers != 1 || d.dirs != 2 || d.mode != kLstm ||
      d.prec != kPrecX3 || T < 8 || N > 16)
    return false;
  if (!pick6(d, N, false) || !use_x3((int)((long)T * N)) || !use_x3(d.nw() * d.H) || !rec6_scratch_free(d, N, false))
    return false;
  return (long)T * N * d.din(0) * 4 < (1L << 31);
}

// ---------------------------------------------------------------------------
// host: backward data (dGates into the reserve, dx)
// ---------------------------------------------------------------------------
int rnn_backward_data(const RnnDesc &d, hipStream_t s, int T, int N, const float *y,
                      const float *dy, const float *w, float *dx, void *workspace,
                      size_t ws_bytes, void *reserve, size_t res_bytes, unsigned *err,
                      hipStream_t overlap, RnnWgradStream *wgrad, const RnnPrepack *pre) {
  RecScope rec_scope;  // the side launches' residency gates (beside_recurrence)
  if (wgrad) wgrad->done = false;
  if (T <= 0 || N <= 0 || N > 16 * kMaxRT || d.H % 16) return KRNN_NOT_SUPPORTED;
  const RnnReserveLayout lay = rnn_reserve_layout(d, T, N);
  if (res_bytes < sizeof(float) * (size_t)lay.total) return KRNN_BAD_PARAM;
  const V6Cfg c6 = pick6(d, N, false);
  const int U6 = c6.U;
  const int U4 = U6 ? 0 : pick_bwd_u4(d, N);
  const int ver = U6 ? 6 : U4 ? 4 : 3;
  const int U = U6 ? U6 : U4 ? U4 : pick_bwd_u(d, N);
  if (d.prec == kPrecBf16 && ver != 6) return KRNN_NOT_SUPPORTED;
  if (!U) return KRNN_NOT_SUPPORTED;
  const int NW = d.nw(), H = d.H, dirs = d.dirs;
  const long TN = (long)T * N;
  float *res = static_cast<float *>(reserve);
  const float *dcur = dy;
  for (int l = d.layers - 1; l >= 0; l--) {
    float *R0 = res + lay.per_layer * l;
    const float *out = (l == d.layers - 1) ? y : R0 + lay.out;
    const int Din = d.din(l);
    const long pl0 = d.lin_offset(l * dirs, 0, false);
    const float *wl = w + pl0;
    const long pls = d.pl_size(l);
    float *E = R0 + lay.E;
    float *DX = d.mode == kGru ? R0 + lay.DX : E;
    if (ver == 3) KCTC_HIP_CHECK(hipMemsetAsync(E, 0xFF, sizeof(float) * TN * dirs * NW * H, s));
    RecParams p{};
    p.T = T; p.N = N; p.H = H; p.dirs = dirs; p.U = U; p.nwg = H / U;
    p.ncol = 16; p.Npad = (N + 15) / 16 * 16;
    p.w = wl; p.pl_stride = pls; p.r_off = d.lin_offset(l * dirs, NW, false) - pl0;
    p.bR_off = d.lin_offset(l * dirs, NW, true) - pl0;
    p.G = R0 + lay.G; p.y = const_cast<float *>(out); p.aux = R0 + lay.aux;
    p.dy = dcur; p.E = E; p.DX = DX; p.bias = R0 + lay.bias; p.err = err;
    p.sync = kSyncFlag;
    p.allow_local = 0;
    if (ws_bytes < rnn_workspace_bytes(d, T, N)) return KRNN_BAD_PARAM;
    p.flags = reinterpret_cast<unsigned *>(static_cast<char *>(workspace) + flags_offset(d, T, N));
    KCTC_HIP_CHECK(hipMemsetAsync(p.flags, 0, kFlagBytes, s));
    const size_t lds = ver == 6 ? bwd6_lds_bytes(d, c6) : bwd_lds_bytes(d, N, U, ver);
    p.xpd = ver == 4 ? v4_xpd(d, U) : 1;
    p.rg = ver == 6 ? c6.rg : 1;
    p.gs = ver == 6 ? c6.gs : 16;
    if (ver == 6) {
      // XCD-pinned backward (xcd_mask): each (row group, direction) on one
      // XCD, the partial-dh hand-off in that XCD's L2, through a ring of two
      // step images (L2-resident).  configs[1]: 3.36 -> 2.70 us per step with
      // the streamed dx GEMM beside it (2.41 without), 468k -> 511k frames/s
      p.xpd = xcd_mask(d, N, false) ? 1 : 0;
      p.ring = p.xpd ? 2 : 0;
      p.allow_local = 1;
      p.poll_sleep = 1;
      p.bfpart = 1;
      p.xch = xch_acquire(sizeof(float) * (size_t)T * dirs * p.nwg * (16 * H + 64) * p.rg, s);
      // self-tagged hand-off (fp32 partials through the L2 ring): the two ring
      // images start with tag 1 in every word (steps 0 and 1 publish tag 0)
      p.dtag = d.prec != kPrecBf16 && p.ring == 2 && p.xpd && T >= 2;
      if (p.dtag)
        KCTC_HIP_CHECK(hipMemsetAsync(p.xch, 0x01, sizeof(float) * 2 * (size_t)dirs * p.nwg * (16 * H + 64) * p.rg, s));
    } else {
      p.xch = reinterpret_cast<float *>(static_cast<char *>(workspace) + xch_offset(d, T, N));
    }
    const dim3 grid(ver == 4 ? 8 * ceil_div(p.nwg, p.xpd) : ver == 6 && p.xpd ? 8 * p.nwg : dirs * p.nwg * p.rg);
    RecTrace tr;
    if (tr.arm("bwd", grid.x)) p.trace = tr.dev;
    // dx_l = sum_dir DX_dir W_dir   (lower layer's dy, or the caller's dx)
    float *dxl = (l == 0) ? dx : res + lay.per_layer * (l - 1) + lay.dout;
    // streamed: computed on `overlap` while the recurrence runs, from its rows as they appear
    const bool streamed = dxl && overlap && ver == 6 && bwd_dx_stream_ok(d, l, T, N);
    // weight gradients streamed off this recurrence (the bottom component):
    // its dGates rows must be written through too
    const bool wstream = wgrad && wgrad->side && !dxl && ver == 6 && !p.xpd && d.layers == 1 &&
                         rnn_wgrad_stream_ok(d, T, N);
    p.e_sc1 = (streamed || wstream) ? 1 : 0;
    // bf16: dGates straight into the packed operands of the dx / dW / dR GEMMs
    // (no fp32 rows, no pack passes over them; KCTC_BF16_DIRECT=0: the fp32
    // rows and the pack kernels as in round 3)
    const bool pkd = bf16_direct(d, ver);  // beside e_sc1's write-through rows when streamed
    if (pkd) {
      p.dxr = reinterpret_cast<__bf16 *>(R0 + lay.pkxr);
      p.dxt = reinterpret_cast<__bf16 *>(R0 + lay.pkxt);
      p.eshift = bf16_io(d) ? 1 : 0;
      p.et = (d.mode == kGru || p.eshift) ? reinterpret_cast<__bf16 *>(R0 + lay.pket) : p.dxt;
      p.kbt64 = lay.kbt64;
      const size_t pitch = sizeof(__bf16) * lay.kbt64;
      const size_t rows = (size_t)NW * H;  // per direction
      if (lay.kbt64 > TN)  // the frame tail of every packed row stays zero
        KCTC_HIP_CHECK(hipMemset2DAsync(p.dxt + TN, pitch, 0, sizeof(__bf16) * (lay.kbt64 - TN), dirs * rows, s));
      if (p.eshift) {  // E^T shifted: direction 0 from TN - N on, direction 1 before N and from TN on
        KCTC_HIP_CHECK(hipMemset2DAsync(p.et + TN - N, pitch, 0, sizeof(__bf16) * (lay.kbt64 - TN + N), rows, s));
        KCTC_HIP_CHECK(hipMemset2DAsync(p.et + rows * lay.kbt64, pitch, 0, sizeof(__bf16) * N, rows, s));
        if (lay.kbt64 > TN)
          KCTC_HIP_CHECK(hipMemset2DAsync(p.et + rows * lay.kbt64 + TN, pitch, 0, sizeof(__bf16) * (lay.kbt64 - TN),
                                          rows, s));
      } else if (d.mode == kGru && lay.kbt64 > TN) {
        KCTC_HIP_CHECK(hipMemset2DAsync(p.et + TN, pitch, 0, sizeof(__bf16) * (lay.kbt64 - TN), dirs * rows, s));
      }
    }
    if (ver == 6) {
      p.cmax = pk<unsigned>(workspace, d, T, N, pack_layout(d, T, N).cme);
      if (p.rg > 1)  // max over the row groups by atomicMax on the float bits
        KCTC_HIP_CHECK(hipMemsetAsync(p.cmax, 0, sizeof(unsigned) * 2 * dirs * NW * H, s));
    }
    const hipEvent_t fork = (streamed || wstream) ? fork_event(s) : nullptr;
    RegWord &rw = reg_of_device();
    if (ver == 6) p.reg = rw.word;  // registration for the exchange's residency gate
    {
      ProfSpan ps(s, "rnn_bwd_rec");
      if (ver == 6) launch6(false, d.mode, d.prec, c6.nth, p, grid, lds, s);
      else launch_rec(false, d.mode, p, grid, lds, s, ver);
    }
    KCTC_HIP_CHECK(hipGetLastError());
    if (ver == 6) {
      // counted once the launch is enqueued (a failed launch never raises the target)
      rw.expected += (unsigned long long)(dirs * p.nwg * p.rg);
      rec_scope.enqueued(p);
      g_last_bwd_scratch_free = rec6_scratch_free(d, N, false);
    } else {
      rec_scope.none();
      g_last_bwd_scratch_free = true;
    }
    if (streamed) {
      launch_bwd_stream(d, p, l, w, dxl, workspace, T, N, overlap, fork, err, d.layers == 1 ? pre : nullptr);
      join_stream(s, overlap);
    }
    if (wstream) {
      // chunk c of C: direction 0 frames [T - b(c+1), T - b(c)), direction 1
      // [b(c), b(c+1)), b(c) = c T / C; complete once every flag line holds
      // epoch b(c+1) + 2 (rows of step k are out at epoch k + 3)
      hipStream_t ws2 = wgrad->side;
      KCTC_HIP_CHECK(hipStreamWaitEvent(ws2, fork, 0));  // after the flag reset
      beside_recurrence(ws2);
      const int C = std::max(1, std::min(wgrad->chunks, T / 4));
      const unsigned *lines = p.flags + 1024;
      const int nlines = p.rg * dirs * p.nwg;
      for (int c = 0; c < C; c++) {
        const int b0 = (int)((long)c * T / C), b1 = (int)((long)(c + 1) * T / C);
        hipLaunchKernelGGL(rec_gate_kernel, dim3(1), dim3(64), 0, ws2, lines, nlines, (unsigned)(b1 + 2), err);
        wgrad_frames(d, ws2, T, N, wgrad->x, y, workspace, wgrad->dw, reserve, wgrad->max_blocks, wgrad->in_bound, 0,
                     T - b1, T - b0);
        wgrad_frames(d, ws2, T, N, wgrad->x, y, workspace, wgrad->dw, reserve, wgrad->max_blocks, wgrad->in_bound, 1,
                     b0, b1);
      }
      join_stream(ws2, s);  // the bias partials are written after the last flag
      wgrad_bias(d, ws2, T, N, wgrad->dw, reserve, 0);
      wgrad->done = true;
    }
    if (ver == 6) xch_release(s);
    tr.dump("bwd", s, grid.x, p.nwg, T, dirs, ver, ver == 6 ? (p.xpd ? 1 : 0) : p.xpd);
    if (dxl && !streamed && d.prec == kPrecBf16 && use_x3(NW * H)) {
      // bf16: dGates rows and W^T rows (columns of W) packed as bf16 (the
      // dGates rows written packed by the recurrence when pkd)
      const long G4 = (long)NW * H;
      const int KB = (int)((G4 + 63) / 64);
      const PackLay pl = pack_layout(d, T, N);
      __bf16 *Ap = pkd ? p.dxr : pk<__bf16>(workspace, d, T, N, pl.a), *Bp = pk<__bf16>(workspace, d, T, N, pl.b);
      {
        ProfSpan ps(s, "x3_pack");
        if (!pkd) bf16_pack_rows(s, DX, (long)dirs * G4, (int)TN, (int)G4, Ap, dirs, G4, TN * KB * 64);
        for (int dir = 0; dir < dirs; dir++)
          bf16_pack_cols(s, wl + dir * pls, Din, (int)G4, Din, 0, Bp + (long)dir * Din * KB * 64);
      }
      for (int dir = 0; dir < dirs; dir++) {
        ProfSpan ps(s, "gemm_bwd_data");
        X3PArgs x;
        x.bf16 = true;
        x.M = (int)TN; x.N = Din; x.KB = KB;
        x.A = reinterpret_cast<const _Float16 *>(Ap + (long)dir * TN * KB * 64);
        x.B = reinterpret_cast<const _Float16 *>(Bp + (long)dir * Din * KB * 64);
        x.C = dxl; x.ldc = Din; x.beta = dir == 0 ? 0.f : 1.f;
        gemm_x3p(s, x);
      }
    } else if (dxl && !streamed) {
      const bool x3 = use_x3(NW * H);
      const long G4 = (long)NW * H;
      const int KB = (int)((G4 + 31) / 32);
      const PackLay pl = pack_layout(d, T, N);
      _Float16 *Ap = pk<_Float16>(workspace, d, T, N, pl.a), *Bp = pk<_Float16>(workspace, d, T, N, pl.b);
      int *eA = pk<int>(workspace, d, T, N, pl.ea), *eB = pk<int>(workspace, d, T, N, pl.eb);
      unsigned *cm = pk<unsigned>(workspace, d, T, N, pl.cm);
      if (x3) {
        // dGates rows (frames, per direction) and W^T rows (input dims), packed over the gates
        ProfSpan ps(s, "x3_pack");
        x3p_pack_rows(s, DX, (long)dirs * G4, (int)TN, (int)G4, Ap, eA, 0.f, dirs, G4, TN * KB * 64, TN);
        for (int dir = 0; dir < dirs; dir++) {
          absmax_f32(s, wl + dir * pls, Din, (int)G4, Din, nullptr, cm);
          x3p_pack_cols(s, wl + dir * pls, Din, (int)G4, Din, 0, Bp + (long)dir * Din * KB * 64, eB + dir * Din, cm,
                        0.f);
        }
      }
      for (int dir = 0; dir < dirs; dir++) {
        ProfSpan ps(s, "gemm_bwd_data");
        if (x3) {
          X3PArgs x;
          x.M = (int)TN; x.N = Din; x.KB = KB;
          x.A = Ap + (long)dir * TN * KB * 64; x.eA = eA + (long)dir * TN;
          x.B = Bp + (long)dir * Din * KB * 64; x.eB = eB + dir * Din;
          x.C = dxl; x.ldc = Din; x.beta = dir == 0 ? 0.f : 1.f;
          gemm_x3p(s, x);
        } else {
          GemmArgs g;
          g.transA = false; g.transB = false;
          g.M = (int)TN; g.N = Din; g.K = NW * H;
          g.A = DX + (long)dir * NW * H; g.lda = (long)dirs * NW * H;
          g.B = wl + dir * pls; g.ldb = Din;
          g.C = dxl; g.ldc = Din;
          g.beta = dir == 0 ? 0.f : 1.f;
          gemm_f32(s, g);
        }
      }
    }
    dcur = dxl;
  }
  return KRNN_OK;
}

// ---------------------------------------------------------------------------
// host: backward weights (accumulates into dw, like cudnnRNNBackwardWeights)
// ---------------------------------------------------------------------------
int rnn_backward_weights(const RnnDesc &d, hipStream_t s, int T, int N, const float *x,
                         const float *y, void *workspace, size_t ws_bytes, float *dw,
                         void *reserve, size_t res_bytes, int max_blocks, float in_bound, hipStream_t s2,
                         const void *in_cols, bool beside, const RnnPrepack *pre) {
  const RnnReserveLayout lay = rnn_reserve_layout(d, T, N);
  if (res_bytes < sizeof(float) * (size_t)lay.total) return KRNN_BAD_PARAM;
  if (ws_bytes < rnn_workspace_bytes(d, T, N)) return KRNN_BAD_PARAM;
  const int NW = d.nw(), H = d.H, dirs = d.dirs, G4 = NW * H;
  const long TN = (long)T * N;
  float *res = static_cast<float *>(reserve);
  float *ws = static_cast<float *>(workspace);
  for (int l = 0; l < d.layers; l++) {
    float *R0 = res + lay.per_layer * l;
    const float *in = l == 0 ? x : res + lay.per_layer * (l - 1) + lay.out;
    const float *out = (l == d.layers - 1) ? y : R0 + lay.out;
    const int Din = d.din(l);
    const long pl0 = d.lin_offset(l * dirs, 0, false);
    const long pls = d.pl_size(l);
    float *dwl = dw + pl0;
    float *E = R0 + lay.E;
    float *DX = d.mode == kGru ? R0 + lay.DX : E;
    const long ldg = (long)dirs * G4, ldy = (long)dirs * H;
    // dW_dir += DX_dir^T x
    GemmArgs g;
    g.transA = true; g.transB = false;
    g.M = G4; g.N = Din; g.K = (int)TN;
    g.A = DX; g.lda = ldg; g.B = in; g.ldb = Din;
    g.C = dwl; g.ldc = Din; g.beta = 1.f;
    g.batch = dirs; g.strideA = G4; g.strideB = 0; g.strideC = pls;
    g.split_k = gemm_pick_split(g.M, g.N, g.K, dirs);
    g.ws = ws;
    g.max_blocks = max_blocks;
    // flag words 1008..1009 of the workspace: dynamic tile counters (the
    // recurrences of this layer, which use the other flag words, are done)
    unsigned *fl = reinterpret_cast<unsigned *>(static_cast<char *>(workspace) + flags_offset(d, T, N));
    if (max_blocks > 0) g.tile_counter = reinterpret_cast<int *>(fl + 1008);
    const bool x3 = use_x3((int)TN);  // K = frames: large (also for a 40-dim input: 0.8 ms/step over fp32)
    if (x3 && d.prec == kPrecBf16) {
      // bf16 weight GEMMs: the transposes packed along the frames as bf16
      const int KB = (int)((TN + 63) / 64);
      const PackLay pl = pack_layout(d, T, N);
      // the dGates transposes: written packed by the backward recurrence (bf16_direct)
      const bool pkd = bf16_direct(d, 6);
      // bf16_io: the forward wrote y^T packed (unshifted) and the backward
      // E^T shifted by one step; the input's columns may come packed from the
      // previous component's forward (in_cols)
      const bool io = bf16_io(d);
      const bool cols_in = l == 0 && in_cols != nullptr;
      __bf16 *DXt = pkd ? reinterpret_cast<__bf16 *>(R0 + lay.pkxt) : pk<__bf16>(workspace, d, T, N, pl.a);
      __bf16 *Xt = cols_in ? static_cast<__bf16 *>(const_cast<void *>(in_cols)) : pk<__bf16>(workspace, d, T, N, pl.b);
      __bf16 *Yt = io ? reinterpret_cast<__bf16 *>(R0 + lay.pkyc) : pk<__bf16>(workspace, d, T, N, pl.c);
      __bf16 *Et = (d.mode == kGru || io)
                       ? (pkd ? reinterpret_cast<__bf16 *>(R0 + lay.pket) : DXt + (long)dirs * G4 * KB * 64)
                       : DXt;
      {
        ProfSpan ps(s, "x3_pack_w");
        if (!pkd) {
          bf16_pack_cols(s, DX, ldg, (int)TN, (int)(dirs * G4), 0, DXt);
          if (d.mode == kGru) bf16_pack_cols(s, E, ldg, (int)TN, (int)(dirs * G4), 0, Et);
        }
        if (!cols_in) bf16_pack_cols(s, in, Din, (int)TN, Din, 0, Xt);
        if (T > 1 && !io)
          for (int dir = 0; dir < dirs; dir++)
            bf16_pack_cols(s, out + (long)dir * H, ldy, (int)TN, H, dir == 0 ? N : -N, Yt + (long)dir * H * KB * 64);
      }
      {
        X3PArgs x;
        x.bf16 = true;
        x.M = (int)G4; x.N = Din; x.KB = KB;
        x.A = reinterpret_cast<const _Float16 *>(DXt); x.sA = G4 * KB * 64;
        x.B = reinterpret_cast<const _Float16 *>(Xt);
        x.C = dwl; x.ldc = Din; x.beta = 1.f;
        x.batch = dirs; x.sC = pls;
        x.split_k = x3p_pick_split((int)G4, Din, KB, dirs); x.ws = ws;
        x.max_blocks = g.max_blocks; x.tile_counter = g.tile_counter;
        ProfSpan ps(s, "gemm_bwd_w");
        gemm_x3p(s, x);
      }
      if (T > 1) {
        X3PArgs x;
        x.bf16 = true;
        x.M = (int)G4; x.N = H; x.KB = KB;
        x.A = reinterpret_cast<const _Float16 *>(Et); x.sA = G4 * KB * 64;
        x.B = reinterpret_cast<const _Float16 *>(Yt); x.sB = (long)H * KB * 64;
        x.C = dwl + (d.lin_offset(l * dirs, NW, false) - pl0); x.ldc = H; x.beta = 1.f;
        x.batch = dirs; x.sC = pls;
        x.split_k = x3p_pick_split((int)G4, H, KB, dirs); x.ws = ws;
        x.max_blocks = max_blocks;
        if (max_blocks > 0) x.tile_counter = reinterpret_cast<int *>(fl + 1009);
        ProfSpan ps(s, "gemm_bwd_r");
        gemm_x3p(s, x);
      }
    }
    if (x3 && d.prec == kPrecBf16) {
    } else {
    const int KBt = (int)((TN + 31) / 32);
    const PackLay pl = pack_layout(d, T, N);
    // x^T and y^T packed by the forward (RnnPrepack::wgrad), else here
    const bool wpre = pre && pre->wdone && pre->wev && use_x3((int)TN) && d.layers == 1 && T > 1;
    _Float16 *DXt = pk<_Float16>(workspace, d, T, N, pl.a);
    _Float16 *Xt = pk<_Float16>(workspace, d, T, N, wpre ? pl.xt : pl.b);
    _Float16 *Yt = pk<_Float16>(workspace, d, T, N, wpre ? pl.yt : pl.c);
    _Float16 *Et = d.mode == kGru ? DXt + (long)dirs * G4 * KBt * 64 : DXt;
    int *eDX = pk<int>(workspace, d, T, N, pl.ea), *eX = pk<int>(workspace, d, T, N, wpre ? pl.ext : pl.eb);
    int *eY = pk<int>(workspace, d, T, N, wpre ? pl.eyt : pl.ec), *eE = d.mode == kGru ? pk<int>(workspace, d, T, N, pl.ed) : eDX;
    if (wpre) KCTC_HIP_CHECK(hipStreamWaitEvent(s, pre->wev, 0));
    unsigned *cm = pk<unsigned>(workspace, d, T, N, pl.cm);
    // two streams (s2, the bottom component's tail, where nothing else
    // overlaps): input^T and output^T are packed and dW runs on s2 while
    // dGates^T is packed and dR runs on s (separate split slabs, tile
    // counters and absmax scratch); s then waits for s2
    const unsigned *cme0 = pick_bwd_u6(d, N) ? pk<unsigned>(workspace, d, T, N, pl.cme) : nullptr;
    // (LSTM: dR's dGates^T is dW's, E == DX; the GRU's E^T pack stays on one stream)
    const bool two = s2 && x3 && cme0 && d.mode == kLstm && d.layers == 1 && T > 1 && env_int("KCTC_WGRAD_2S", 1);
    hipStream_t sx = two ? s2 : s;  // stream of the input / output packs and of dW
    hipEvent_t ev_dx = nullptr, ev_y = nullptr;
    if (two) {
      KCTC_HIP_CHECK(hipEventCreateWithFlags(&ev_dx, hipEventDisableTiming));
      KCTC_HIP_CHECK(hipEventCreateWithFlags(&ev_y, hipEventDisableTiming));
      join_stream(s2, s);
    }
    if (two) {
      ProfSpan ps(s, "x3_pack_w");
      x3p_pack_cols(s, DX, ldg, (int)TN, (int)(dirs * G4), 0, DXt, eDX, cme0, 0.f);
      KCTC_HIP_CHECK(hipEventRecord(ev_dx, s));
      const bool xb = l == 0 && in_bound > 0.f;
      // absmax scratch of its own: the GRU-only E^T exponent array (free for an LSTM)
      unsigned *cmx = reinterpret_cast<unsigned *>(pk<int>(workspace, d, T, N, pl.ed));
      if (!wpre) {
        if (!xb) absmax_f32(s2, in, Din, (int)TN, Din, nullptr, cmx);
        x3p_pack_cols(s2, in, Din, (int)TN, Din, 0, Xt, eX, cmx, xb ? in_bound : 0.f);
        for (int dir = 0; dir < dirs; dir++)
          x3p_pack_cols(s2, out + (long)dir * H, ldy, (int)TN, H, dir == 0 ? N : -N, Yt + (long)dir * H * KBt * 64,
                        eY + dir * H, nullptr, 1.f);
      }
      KCTC_HIP_CHECK(hipEventRecord(ev_y, s2));
      KCTC_HIP_CHECK(hipStreamWaitEvent(s2, ev_dx, 0));
      KCTC_HIP_CHECK(hipStreamWaitEvent(s, ev_y, 0));
    } else if (x3) {
      // the transposes, packed over the frames: dGates^T (per-gate exponents),
      // input^T (per-dim), and for dR the output shifted by one step per direction
      ProfSpan ps(s, "x3_pack_w");
      // beside a pinned recurrence: off its XCDs (x3p_pack_cols avoid)
      const unsigned *av = beside ? rnn_pinned_xcds() : nullptr;
      const int nx = std::max(1, rnn_usable_cus() / kCusPerXcd);
      // their item counters: flag words 1010..1014 (this component's
      // recurrences, which use the flag words, are done)
      int *pc = reinterpret_cast<int *>(fl + 1010);
      if (av) KCTC_HIP_CHECK(hipMemsetAsync(pc, 0, sizeof(int) * 5, s));
      // the v6 backward recurrence leaves the dGates column maxima behind
      const unsigned *cme = cme0;
      if (!cme) absmax_f32(s, DX, ldg, (int)TN, (int)(dirs * G4), nullptr, cm);
      x3p_pack_cols(s, DX, ldg, (int)TN, (int)(dirs * G4), 0, DXt, eDX, cme ? cme : cm, 0.f, 1, 0, 0, 0, 0, av, nx,
                    pc);
      if (d.mode == kGru) {
        if (!cme) absmax_f32(s, E, ldg, (int)TN, (int)(dirs * G4), nullptr, cm);
        x3p_pack_cols(s, E, ldg, (int)TN, (int)(dirs * G4), 0, Et, eE, cme ? cme + dirs * G4 : cm, 0.f, 1, 0, 0, 0,
                      0, av, nx, pc + 1);
      }
      const bool xb = (l > 0 && bounded_out(d)) || (l == 0 && in_bound > 0.f);
      if (!xb && !wpre) absmax_f32(s, in, Din, (int)TN, Din, nullptr, cm);
      if (!wpre)
        x3p_pack_cols(s, in, Din, (int)TN, Din, 0, Xt, eX, cm, xb ? (l > 0 ? 1.f : in_bound) : 0.f, 1, 0, 0, 0, 0,
                      av, nx, pc + 2);
      if (T > 1 && !wpre) {
        if (!bounded_out(d)) absmax_f32(s, out, ldy, (int)TN, (int)ldy, nullptr, cm);
        for (int dir = 0; dir < dirs; dir++)
          x3p_pack_cols(s, out + (long)dir * H, ldy, (int)TN, H, dir == 0 ? N : -N, Yt + (long)dir * H * KBt * 64,
                        eY + dir * H, bounded_out(d) ? nullptr : cm + dir * H, bounded_out(d) ? 1.f : 0.f, 1, 0, 0,
                        0, 0, av, nx, pc + 3 + dir);
      }
    }
    // beside another component's pinned backward recurrence: dW and dR as
    // one launch on the CUs it leaves (gemm_x3p_pair; configs[1]: the side
    // stream fell one GEMM per layer behind, 4 ms of weight GEMMs after the
    // last recurrence)
    const bool pair = beside && x3 && !two && T > 1 && x3p_use_256((int)G4, Din) && x3p_use_256((int)G4, H) &&
                      max_blocks > 0;
    X3PArgs xw;
    if (x3) {
      X3PArgs &x = xw;
      x.M = (int)G4; x.N = Din; x.KB = KBt;
      x.A = DXt; x.eA = eDX; x.sA = G4 * KBt * 64; x.seA = G4;
      x.B = Xt; x.eB = eX;
      x.C = dwl; x.ldc = Din; x.beta = 1.f;
      x.batch = dirs; x.sC = pls;
      x.split_k = x3p_pick_split((int)G4, Din, KBt, dirs);
      // concurrent with dR: its own split slab past dR's (none when dR is not
      // split: drec_split_floats reserves a dR slab only for a split > 1)
      const long sR = x3p_pick_split((int)G4, H, KBt, dirs);
      x.ws = (two || pair) && sR > 1 ? ws + al64(sR * dirs * G4 * H) : ws;
      x.max_blocks = g.max_blocks; x.tile_counter = g.tile_counter;
      if (pair) {
        x.max_blocks = 192;
        x.avoid_word = rnn_pinned_xcds();
        x.avoid_xcds = std::max(1, rnn_usable_cus() / kCusPerXcd);
      } else {
        ProfSpan ps(sx, "gemm_bwd_w");
        gemm_x3p(sx, x);
      }
    } else {
      ProfSpan ps(s, "gemm_bwd_w");
      gemm_f32(s, g);
    }
    // dR_dir += E_dir(shifted)^T h_prev:  fwd pairs rows t>=1 with y rows t-1,
    // bwd pairs rows t<=T-2 with y rows t+1 (column half H..2H-1)
    if (T > 1) {
      GemmArgs r;
      r.transA = true; r.transB = false;
      r.M = G4; r.N = H; r.K = (int)((long)(T - 1) * N);
      r.A = E + (long)N * ldg; r.lda = ldg;
      r.B = out; r.ldb = ldy;
      r.C = dwl + (d.lin_offset(l * dirs, NW, false) - pl0); r.ldc = H; r.beta = 1.f;
      r.batch = dirs;
      r.strideA = (long)G4 - (long)N * ldg;        // dir 1: E + G4 (rows 0..T-2)
      r.strideB = (long)N * ldy + H;               // dir 1: y rows 1..T-1, cols H..
      r.strideC = pls;
      r.split_k = gemm_pick_split(r.M, r.N, r.K, dirs);
      r.ws = ws;
      r.max_blocks = max_blocks;
      if (max_blocks > 0) r.tile_counter = reinterpret_cast<int *>(fl + 1009);
      ProfSpan ps(s, "gemm_bwd_r");
      if (x3) {
        // all frames: the shifted-out ones are zero in the packed output
        X3PArgs x;
        x.M = (int)G4; x.N = H; x.KB = KBt;
        x.A = Et; x.eA = eE; x.sA = G4 * KBt * 64; x.seA = G4;
        x.B = Yt; x.eB = eY; x.sB = (long)H * KBt * 64; x.seB = H;
        x.C = r.C; x.ldc = H; x.beta = 1.f;
        x.batch = dirs; x.sC = pls;
        x.split_k = x3p_pick_split((int)G4, H, KBt, dirs); x.ws = ws;
        x.max_blocks = max_blocks; x.tile_counter = r.tile_counter;
        if (pair) gemm_x3p_pair(s, xw, x);  // xw's tile counter, block count and avoid word
        else gemm_x3p(s, x);
      } else {
        gemm_f32(s, r);
      }
    }
    if (two) {
      join_stream(s, s2);
      (void)hipEventDestroy(ev_dx);
      (void)hipEventDestroy(ev_y);
    }
    }  // x3 / fp32 weight GEMMs
    // biases: dbW += sum dGx, dbR += sum dGh (partials from the recurrence)
    const long bW = d.lin_offset(l * dirs, 0, true) - pl0;
    const long bR = d.lin_offset(l * dirs, NW, true) - pl0;
    // (v6: one partial per row group, [group][dir][2][G], added in group order)
    const V6Cfg c6b = pick6(d, N, false);
    const int rg = c6b ? c6b.rg : 1;
    for (int gi = 0; gi < rg; gi++)
      for (int dir = 0; dir < dirs; dir++) {
        const float *part = R0 + lay.bias + ((long)gi * dirs + dir) * 2 * G4;
        clip_sgd_update(s, dwl + dir * pls + bW, part, G4, 1.f, 0.f);
        clip_sgd_update(s, dwl + dir * pls + bR, part + G4, G4, 1.f, 0.f);
      }
  }
  return KRNN_OK;
}

}  // namespace kctc
