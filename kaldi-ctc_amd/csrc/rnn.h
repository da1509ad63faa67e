// rnn.h -- cuDNN-v5-compatible recurrent layer on gfx950 (internal C++ API).
// Replaces cudnnRNNForwardTraining / BackwardData / BackwardWeights as wrapped
// by src/cudamatrix/cudnn-recurrent.cc:13-102 of the reference.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace kctc {

enum RnnMode { kRelu = 0, kTanh = 1, kLstm = 2, kGru = 3 };

inline int rnn_nw(int mode) { return mode == kLstm ? 4 : mode == kGru ? 3 : 1; }

struct RnnDesc {
  int mode = kLstm, D = 0, H = 0, layers = 1, dirs = 2;
  // products of the recurrences and gate GEMMs: 0 fp32-class (split-fp16
  // pairs, fp32 accumulation), 1 bf16 (fp32 accumulation, fp32 master weights)
  int prec = 0;
  // bf16 only, latched by rnn_set_precision (not re-read per call: the reserve
  // layout must not change between the size query, the forward and the
  // backward): the recurrences write their GEMM operands packed (pk) and, one
  // layer bidirectional, the forward its output too (pkio)
  int pk = 1, pkio = 1;
  int nw() const { return rnn_nw(mode); }
  int din(int layer) const { return layer == 0 ? D : dirs * H; }
  // floats of one pseudo-layer block [W | R | bW | bR] of stacked layer `layer`
  long pl_size(int layer) const {
    long n = nw();
    return n * H * (long)din(layer) + n * H * (long)H + 2 * n * H;
  }
  long params_size() const;
  // float offset of lin layer `lin` (matrix or bias) of pseudo-layer p = layer*dirs + dir
  long lin_offset(int p, int lin, bool bias) const;
};

// Per-layer regions of the training reserve (floats), kept from forward to
// backward exactly like cuDNN's reserveSpace.
struct RnnReserveLayout {
  long G, aux, E, DX, bias, out, dout, per_layer, total;
  // bf16 precision: the backward recurrence's packed bf16 dGates operands
  // (RecParams::dxr / dxt / et; float offsets, 0 bytes otherwise), frames
  // padded to kbt64 per packed row
  long pkxr, pkxt, pket, kbt64;
  // bf16, one layer, bidirectional: the forward's packed bf16 copies of its
  // output (rows [T*N][2H], columns [2H][kbt64]); see rnn_packed_output
  long pkyr, pkyc;
};
RnnReserveLayout rnn_reserve_layout(const RnnDesc &d, int T, int N);
// set d.prec and latch the packed-operand switches (KCTC_BF16_DIRECT /
// KCTC_BF16_IO, both on by default) into d.pk / d.pkio
void rnn_set_precision(RnnDesc &d, int prec);
size_t rnn_workspace_bytes(const RnnDesc &d, int T, int N);

// CU budget of the persistent kernels.  A v6 recurrence needs
// all of its workgroups resident at once (one per CU, >= 96 KB LDS) and the
// streamed GEMMs' persistent blocks (one per CU as well) spin on its flags,
// so everything that may hold a CU beside them has to fit:
//   recurrence WGs + streamed blocks + comm CUs + 16 (margin) <= usable CUs.
// `cus`: the CUs this process may use (0: the device's; a smaller number
// when ranks share a device through CU-masked streams); `comm`: CUs the
// gradient exchange's kernels (RCCL, capped by maxCTAs) may hold during a
// backward pass.  Streaming is switched off when fewer than 8 blocks fit.
void rnn_set_cu_budget(int cus, int comm);
int rnn_usable_cus();
int rnn_comm_cus();

// Residency gate of the gradient exchange.  Every workgroup
// of a v6 backward recurrence adds 1 to a per-device 64-bit registration
// counter when it starts; rnn_bwd_registrations() is the value it reaches
// once all backward recurrences enqueued so far on this device are resident.
// rnn_comm_gate(s, target) enqueues on s a gate kernel that returns once the
// counter has reached `target` (after 10 s it gives up and flags a gate
// timeout in the device word).  A gate is 8 one-wave blocks, one per XCD;
// a block on an XCD a recurrence is pinned to leaves (unless it is the last
// one waiting), so that no gate wave holds a CU a workgroup of that
// recurrence needs -- a workgroup that takes a CU's whole register file
// cannot be placed beside one (rnn.hip gate_kernel).  An exchange
// that runs its kernels only behind such a gate -- i.e. only while the
// backward recurrence launched last is fully resident -- and makes the next
// recurrence launch wait for them declares rnn_set_comm_gated(true): the
// backward recurrences then stay XCD-pinned with an exchange configured.
unsigned long long rnn_bwd_registrations();
// false when the backward recurrence this thread enqueued last uses scratch:
// nothing may then be queued beside it (rnn.hip rec6_scratch_free), so the
// exchange waits for its end instead of its residency
bool rnn_last_bwd_scratch_free();
void rnn_comm_gate(hipStream_t s, unsigned long long target);
// s waits until the v6 launch whose flag area is `flags` has `target`
// workgroups resident (its own residency count; the same gate kernel, its
// blocks leaving on the XCDs that launch runs on)
void rnn_resident_gate(hipStream_t s, const unsigned *flags, unsigned target);
// Launches beside a running recurrence.  Every v6 recurrence counts its
// resident workgroups in its own flag area (kResWord, zeroed with the flags
// before the launch).  Each kernel that rnn.hip puts on another stream while
// that recurrence runs -- the streamed GEMMs, the wgrad chunk gates, the
// forward-time packs -- is enqueued behind a gate kernel waiting for that count
// (rnn.hip beside_recurrence): nothing there can take a CU before every
// workgroup of the recurrence holds its own, so a consumer spinning on the
// recurrence's progress cannot keep a producer workgroup out.  The host
// refuses a streaming launch (gemm_x3p with stream_flags,
// gemm_x3p_bwd_stream) on a stream that has not passed the gate of the
// recurrence this thread has in flight: rnn_side_gated(s) is false then.
bool rnn_side_gated(hipStream_t s);
// device word: bit x set once an XCD-pinned backward recurrence ran on XCD x
// (never cleared; GEMMs launched beside one avoid those XCDs, X3PArgs::avoid_word)
const unsigned *rnn_pinned_xcds();
void rnn_set_comm_gated(bool on);
bool rnn_comm_gated();

// Status codes of the RNN ABI (include/kaldi_rnn.h)
enum { KRNN_OK = 0, KRNN_BAD_PARAM = 1, KRNN_NOT_SUPPORTED = 2, KRNN_EXEC_FAILED = 3,
       KRNN_TIMEOUT = 4 };

// All calls are stream-ordered; `err` is a device word (0 = ok) that the
// persistent kernels set on a bounded-spin timeout.
// Forward chaining of stacked components: the NEXT RNN component's layer-0
// input projection (the x3 GEMM of this call's output y) is computed on
// `side` while this call's last recurrence is still running, reading the
// recurrence's exchange images in place as their rows get published
// (gemm_x3p streaming mode).  The fork / join with `s` happens inside; `done`
// tells the caller whether the chain was taken -- if so it passes
// input_projected = true to the next component's forward, which then skips
// its layer-0 projection.
struct RnnFwdChain {
  const RnnDesc *d = nullptr;   // the consumer
  const float *w = nullptr;     // its parameters
  void *workspace = nullptr;    // its workspace / reserve (rnn_workspace_bytes, rnn_reserve_layout)
  size_t ws_bytes = 0;
  void *reserve = nullptr;
  size_t res_bytes = 0;
  hipStream_t side = nullptr;
  bool done = false;
};
// in_rows (nullable): the input already packed as bf16 rows [T*N][D] (the
// previous component's rnn_packed_output), used by a bf16 input projection
// instead of packing x.
// The backward's streamed dx GEMM reads W's columns packed (split-fp16 /
// bf16 rows of W^T).  W does not change between a training step's forward and
// backward, so rnn_forward_training packs them on `stream` while its own
// recurrence runs (CUs it leaves idle) into the workspace and records `ev`;
// rnn_backward_data then starts its streamed GEMM at once instead of behind
// the packs.  The caller owns ev and passes the same struct to the backward
// only while the parameters are unchanged (done: set by the forward).
struct RnnPrepack {
  hipStream_t stream = nullptr;
  hipEvent_t ev = nullptr;
  bool done = false;
  // the weight GEMMs' input^T and output^T (x and y packed along the frames,
  // one-layer split-fp16 components with bounded x and y): packed on `stream`
  // by the forward -- x beside its recurrence, y after it -- instead of on the
  // backward's side stream, where the CUs beside the next component's
  // recurrence are short (wev: recorded after both; wdone: packed)
  hipEvent_t wev = nullptr;
  bool dx = true;        // W^T (ev / done) requested
  bool wgrad = false;    // requested
  float in_bound = 0.f;  // |x| <= in_bound (> 0 required)
  bool wdone = false;
};
int rnn_forward_training(const RnnDesc &d, hipStream_t s, int T, int N, const float *x,
                         const float *w, float *y, void *workspace, size_t ws_bytes,
                         void *reserve, size_t res_bytes, unsigned *err, RnnFwdChain *chain = nullptr,
                         bool input_projected = false, const void *in_rows = nullptr, RnnPrepack *pre = nullptr);
// bf16 one-layer bidirectional components: the forward recurrence also writes
// its output as packed bf16 rows [T*N][2H] and columns [2H][kbt64] into the
// reserve (the GEMM operands the next component's projection / dW and this
// component's dR read).  Pointers valid after rnn_forward_training of (T, N)
// on this reserve; false (nullptrs) for other components.
bool rnn_packed_output(const RnnDesc &d, int T, int N, void *reserve, const void **rows, const void **cols);
// Weight gradients of a one-layer bidirectional split-fp16 LSTM computed off
// its RUNNING backward recurrence (the bottom component, which has no dx to
// stream): the frames are cut into `chunks` per direction in the order the
// recurrence finishes them (direction 0 from the last frame down, direction
// 1 from the first up); on `side`, a one-wave gate kernel waits for the
// recurrence's flags to pass a chunk, then that chunk's transposes are packed
// and its dW / dR GEMMs accumulate (beta = 1) into dw; the bias sums follow
// the recurrence.  `dw` must be zeroed on `side` before.  done = launched.
struct RnnWgradStream {
  hipStream_t side = nullptr;
  int chunks = 4;
  const float *x = nullptr;  // the layer input
  float *dw = nullptr;       // gradient (cuDNN layout)
  int max_blocks = 0;
  float in_bound = 0.f;
  bool done = false;
};
bool rnn_wgrad_stream_ok(const RnnDesc &d, int T, int N);
int rnn_backward_data(const RnnDesc &d, hipStream_t s, int T, int N, const float *y,
                      const float *dy, const float *w, float *dx, void *workspace,
                      size_t ws_bytes, void *reserve, size_t res_bytes, unsigned *err,
                      hipStream_t overlap = nullptr,  // overlap: stream for the streamed dx GEMM
                      RnnWgradStream *wgrad = nullptr,
                      const RnnPrepack *pre = nullptr);  // W^T packed by the forward (done)
int rnn_backward_weights(const RnnDesc &d, hipStream_t s, int T, int N, const float *x,
                         const float *y, void *workspace, size_t ws_bytes, float *dw,
                         void *reserve, size_t res_bytes, int max_blocks = 0,
                         float in_bound = 0.f,  // > 0: |x| <= in_bound (an LSTM/GRU below)
                         hipStream_t s2 = nullptr,  // second stream: dW beside dR (nothing else to overlap)
                         const void *in_cols = nullptr,  // bf16: x packed as columns (rnn_packed_output)
                         // runs beside another component's backward recurrence
                         // (the side stream): dW and dR as one launch, kept
                         // off the XCDs pinned recurrences run on
                         bool beside = false,
                         const RnnPrepack *pre = nullptr);  // wdone: x^T / y^T packed by the forward

}  // namespace kctc
