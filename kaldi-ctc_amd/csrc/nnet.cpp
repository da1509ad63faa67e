// nnet.cpp -- nnet2 CTC training path on MI355X (see nnet.h for the mapping to
// the reference's classes).
#include "nnet.h"
#include "kaldi_io.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <sstream>

#include "common.h"
#include "ctc.h"
#include "decodable.h"
#include "elementwise.h"
#include "gemm.h"
#include "prof.h"

namespace kctc {
namespace nnet2 {

// Unit-cost Levenshtein distance (kaldi::LevenshteinEditDistance,
// src/util/edit-distance-inl.h) by Myers' bit-vector algorithm in its block
// form (Myers 1999; the per-block step as in edlib): column j of the DP over
// ref (rows, 64 per word) is kept as vertical +1/-1 delta masks; one pass per
// hyp symbol costs ceil(m/64) word steps instead of m cell updates.  The
// horizontal delta at the top boundary is +1 (D[0][j] = j); bits above row
// m-1 in the last word never reach lower rows (carries and shifts go up).
int levenshtein(const int *ref, int m, const int *hyp, int n) {
  if (m <= 0) return n > 0 ? n : 0;
  if (n <= 0) return m;
  const int W = (m + 63) / 64;
  int lo = ref[0], hi = ref[0];
  for (int i = 1; i < m; i++) { lo = std::min(lo, ref[i]); hi = std::max(hi, ref[i]); }
  std::vector<uint64_t> peq((size_t)(hi - lo + 2) * W, 0);  // last row: symbols absent from ref
  for (int i = 0; i < m; i++) peq[(size_t)(ref[i] - lo) * W + i / 64] |= 1ull << (i % 64);
  std::vector<uint64_t> P(W, ~0ull), M(W, 0ull);
  const uint64_t last = 1ull << ((m - 1) % 64);
  int score = m;
  for (int j = 0; j < n; j++) {
    const int c = hyp[j];
    const uint64_t *eq = &peq[(size_t)((c >= lo && c <= hi) ? c - lo : hi - lo + 1) * W];
    int hin = 1;
    for (int b = 0; b < W; b++) {
      const uint64_t Pv = P[b], Mv = M[b], hneg = hin < 0 ? 1ull : 0ull;
      uint64_t Eq = eq[b];
      const uint64_t Xv = Eq | Mv;
      Eq |= hneg;
      const uint64_t Xh = (((Eq & Pv) + Pv) ^ Pv) | Eq;
      uint64_t Ph = Mv | ~(Xh | Pv);
      uint64_t Mh = Pv & Xh;
      const uint64_t hb = b == W - 1 ? last : (1ull << 63);
      const int hout = (Ph & hb) ? 1 : ((Mh & hb) ? -1 : 0);
      Ph = (Ph << 1) | (hin > 0 ? 1ull : 0ull);
      Mh = (Mh << 1) | hneg;
      P[b] = Mh | ~(Xv | Ph);
      M[b] = Ph & Xv;
      hin = hout;
    }
    score += hin;
  }
  return score;
}

// ---------------------------------------------------------------------------
// plumbing
// ---------------------------------------------------------------------------
DevBuf::~DevBuf() {
  if (p) (void)hipFree(p);
}

void DevBuf::ensure(size_t b) {
  if (b <= bytes && p) return;
  if (p) {
    auto &d = CuDevice::Instantiate();
    KCTC_HIP_CHECK(hipStreamSynchronize(d.stream));
    if (d.side) KCTC_HIP_CHECK(hipStreamSynchronize(d.side));
    if (d.stream2) KCTC_HIP_CHECK(hipStreamSynchronize(d.stream2));
    KCTC_HIP_CHECK(hipFree(p));
    p = nullptr;
  }
  size_t nb = align_up(std::max<size_t>(b, 256), 4096);
  KCTC_HIP_CHECK(hipMalloc(&p, nb));
  // zeroed before any use (flag words that hold ids, e.g. the gated
  // projection's tile flags, must not start out as one by chance)
  KCTC_HIP_CHECK(hipMemsetAsync(p, 0, nb, nullptr));
  KCTC_HIP_CHECK(hipStreamSynchronize(nullptr));
  bytes = nb;
}

void CuMatrix::Resize(long rows, int cols) {
  buf_.ensure(sizeof(float) * (size_t)std::max<long>(1, rows * (long)cols));
  data_ = buf_.f();
  rows_ = rows;
  cols_ = cols;
}

CuDevice &CuDevice::Instantiate() {
  static thread_local CuDevice dev;
  return dev;
}

void CuDevice::Fork() {
  if (!side) return;
  if (!fork_ev) KCTC_HIP_CHECK(hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming));
  KCTC_HIP_CHECK(hipEventRecord(fork_ev, stream));
  KCTC_HIP_CHECK(hipStreamWaitEvent(side, fork_ev, 0));
}

void CuDevice::Join() {
  if (!side) return;
  if (!join_ev) KCTC_HIP_CHECK(hipEventCreateWithFlags(&join_ev, hipEventDisableTiming));
  KCTC_HIP_CHECK(hipEventRecord(join_ev, side));
  KCTC_HIP_CHECK(hipStreamWaitEvent(stream, join_ev, 0));
}

void CuDevice::Begin(const char *family, hipStream_t s) {
  if (!profiling) return;
  if (!s) s = stream;
  if (pool.size() < 2) {
    for (int i = 0; i < 64; i++) {
      hipEvent_t e;
      KCTC_HIP_CHECK(hipEventCreate(&e));
      pool.push_back(e);
    }
  }
  Span sp;
  sp.family = family;
  sp.a = pool.back(); pool.pop_back();
  sp.b = pool.back(); pool.pop_back();
  sp.s = s;
  KCTC_HIP_CHECK(hipEventRecord(sp.a, s));
  open.push_back(spans.size());
  spans.push_back(sp);
}

void CuDevice::End() {
  if (!profiling || open.empty()) return;
  KCTC_HIP_CHECK(hipEventRecord(spans[open.back()].b, spans[open.back()].s));
  open.pop_back();
}

void CuDevice::Collect() {
  for (auto &sp : spans) {
    float ms = 0.f;
    KCTC_HIP_CHECK(hipEventElapsedTime(&ms, sp.a, sp.b));
    auto &e = prof[sp.family];
    e.first += ms;
    e.second += 1;
    pool.push_back(sp.a);
    pool.push_back(sp.b);
  }
  spans.clear();
}

}  // namespace nnet2

void prof_begin(hipStream_t s, const char *family) {
  auto &d = nnet2::CuDevice::Instantiate();
  if (d.profiling && (s == d.stream || (s && s == d.side))) d.Begin(family, s);
}
void prof_end(hipStream_t s) {
  auto &d = nnet2::CuDevice::Instantiate();
  if (d.profiling && (s == d.stream || (s && s == d.side))) d.End();
}

namespace nnet2 {

struct ProfScope {
  explicit ProfScope(const char *f, hipStream_t s = nullptr) { CuDevice::Instantiate().Begin(f, s); }
  ~ProfScope() { CuDevice::Instantiate().End(); }
};

uint64_t Rng::next() {
  uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
double Rng::uniform() { return ((double)(next() >> 11) + 0.5) * (1.0 / 9007199254740992.0); }
double Rng::gauss() {
  const double u1 = uniform(), u2 = uniform();
  return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
}

static hipStream_t S() { return CuDevice::Instantiate().stream; }

// ---- config parsing: ParseFromString (src/nnet2/nnet-component.cc:160-260) ----
static std::vector<std::string> split_ws(const std::string &s) {
  std::vector<std::string> out;
  std::istringstream is(s);
  std::string t;
  while (is >> t) out.push_back(t);
  return out;
}

static bool take(const std::string &name, std::string *args, std::string *val) {
  auto parts = split_ws(*args);
  const std::string ne = name + "=";
  for (size_t i = 0; i < parts.size(); i++) {
    if (parts[i].compare(0, ne.size(), ne) == 0) {
      *val = parts[i].substr(ne.size());
      std::string rest;
      for (size_t j = 0; j < parts.size(); j++)
        if (j != i) rest += (rest.empty() ? "" : " ") + parts[j];
      *args = rest;
      return true;
    }
  }
  return false;
}
static bool ParseFromString(const std::string &name, std::string *args, int *v) {
  std::string s;
  if (!take(name, args, &s)) return false;
  char *end = nullptr;
  long x = strtol(s.c_str(), &end, 10);
  if (s.empty() || *end) throw std::invalid_argument("Bad option " + name + "=" + s);
  *v = (int)x;
  return true;
}
static bool ParseFromString(const std::string &name, std::string *args, float *v) {
  std::string s;
  if (!take(name, args, &s)) return false;
  char *end = nullptr;
  double x = strtod(s.c_str(), &end);
  if (s.empty() || *end) throw std::invalid_argument("Bad option " + name + "=" + s);
  *v = (float)x;
  return true;
}
static bool ParseFromString(const std::string &name, std::string *args, bool *v) {
  std::string s;
  if (!take(name, args, &s)) return false;
  if (s.empty()) throw std::invalid_argument("Bad option " + name);
  if (s[0] == 'f' || s[0] == 'F') *v = false;
  else if (s[0] == 't' || s[0] == 'T') *v = true;
  else throw std::invalid_argument("Bad option " + name + "=" + s);
  return true;
}
static bool ParseFromString(const std::string &name, std::string *args, std::vector<int> *v) {
  std::string s;
  if (!take(name, args, &s)) return false;
  v->clear();
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, ':')) v->push_back(std::stoi(tok));
  return true;
}

// ---- Kaldi token stream, both modes (kaldi_io.h) ----
using kio::ExpectToken;
using kio::WriteToken;
// counters are int32 in the reference's files (nnet-cudnn-component.h:263-266)
static int32_t as_i32(double v) { return (int32_t)(uint32_t)(uint64_t)(int64_t)v; }
static std::vector<float> d2h(const float *d, long n) {
  std::vector<float> h((size_t)n);
  if (n) {
    KCTC_HIP_CHECK(hipMemcpyAsync(h.data(), d, sizeof(float) * n, hipMemcpyDeviceToHost, S()));
    KCTC_HIP_CHECK(hipStreamSynchronize(S()));
  }
  return h;
}
static void h2d(float *d, const float *h, long n) {
  if (!n) return;
  KCTC_HIP_CHECK(hipMemcpyAsync(d, h, sizeof(float) * n, hipMemcpyHostToDevice, S()));
  KCTC_HIP_CHECK(hipStreamSynchronize(S()));
}

std::string Component::Info() const {
  std::ostringstream os;
  os << Type() << ", input-dim=" << InputDim() << ", output-dim=" << OutputDim();
  return os.str();
}

Component *Component::NewComponentOfType(const std::string &type) {
  if (type == "SpliceComponent") return new SpliceComponent;
  if (type == "CuDNNRecurrentComponent") return new CuDNNRecurrentComponent;
  if (type == "ClipGradientComponent") return new ClipGradientComponent;
  if (type == "AffineComponent") return new AffineComponent;
  if (type == "SoftmaxComponent") return new SoftmaxComponent;
  return nullptr;
}

Component *Component::ReadNew(std::istream &is, bool binary) {
  const std::string t = kio::ReadToken(is, binary);
  if (t.size() < 3 || t.front() != '<' || t.back() != '>') throw std::runtime_error("bad component token " + t);
  Component *c = NewComponentOfType(t.substr(1, t.size() - 2));
  if (!c) throw std::runtime_error("Unknown component type " + t);
  try {
    c->Read(is, binary);
  } catch (...) {
    delete c;
    throw;
  }
  return c;
}

// ---------------------------------------------------------------------------
// SpliceComponent (nnet-component.cc:2504-2820)
// ---------------------------------------------------------------------------
void SpliceComponent::Init(int input_dim, std::vector<int> context, int const_dim) {  // :2504-2513
  if (context.empty() || input_dim <= 0 || context.front() > 0 || context.back() < 0)
    throw std::invalid_argument("SpliceComponent: context must contain offsets <= 0 and >= 0");
  for (size_t i = 1; i < context.size(); i++)
    if (context[i] <= context[i - 1]) throw std::invalid_argument("SpliceComponent: context must be sorted and unique");
  if (const_dim < 0 || const_dim >= input_dim) throw std::invalid_argument("SpliceComponent: bad const-component-dim");
  input_dim_ = input_dim;
  context_ = std::move(context);
  const_dim_ = const_dim;
}
void SpliceComponent::InitFromString(std::string args, Rng &) {  // :2517-2540
  const std::string orig = args;
  int input_dim = 0, left = 0, right = 0, cdim = 0;
  std::vector<int> context;
  bool in_ok = ParseFromString("input-dim", &args, &input_dim);
  bool ctx_ok = ParseFromString("context", &args, &context);
  bool lr_ok = ParseFromString("left-context", &args, &left) &&
               ParseFromString("right-context", &args, &right);
  ParseFromString("const-component-dim", &args, &cdim);
  if (!(in_ok && (ctx_ok || lr_ok)) || !args.empty() || input_dim <= 0)
    throw std::invalid_argument("Invalid initializer for layer of type SpliceComponent: \"" + orig + "\"");
  if (lr_ok) {
    if (!context.empty()) throw std::invalid_argument("SpliceComponent: context and left/right-context both given");
    for (int i = -left; i <= right; i++) context.push_back(i);
  }
  Init(input_dim, context, cdim);
}
void SpliceComponent::Propagate(const ChunkInfo &in_info, const ChunkInfo &out_info, const CuMatrixBase &in,
                                CuMatrixBase *out) const {
  if (IsIdentityForward()) {
    if (out->Data() != in.Data())
      KCTC_HIP_CHECK(hipMemcpyAsync(out->Data(), in.Data(), sizeof(float) * in.NumRows() * in.NumCols(),
                                    hipMemcpyDeviceToDevice, S()));
    return;
  }
  const long rows = out->NumRows();
  if (rows <= 0 || in.NumRows() % rows) throw std::invalid_argument("SpliceComponent: input rows are not chunks of the output rows");
  const int ns = (int)(in.NumRows() / rows);
  // input row of output frame j for context offset 0: j * ns + (out offset - in offset)
  const int first = out_info.first_offset - in_info.first_offset;
  if (first + context_.front() < 0 || first + context_.back() >= ns)
    throw std::invalid_argument("SpliceComponent: context outside the input chunk");
  splice_rows(S(), in.Data(), input_dim_, ns, rows, context_.data(), (int)context_.size(), first, const_dim_,
              out->Data());
}
void SpliceComponent::Backprop(const ChunkInfo &in_info, const ChunkInfo &out_info, const CuMatrixBase &,
                               const CuMatrixBase &, const CuMatrixBase &out_deriv, Component *,
                               CuMatrixBase *in_deriv) const {  // :2691-2760
  if (!in_deriv) return;
  if (IsIdentityForward()) {
    if (in_deriv->Data() != out_deriv.Data())
      KCTC_HIP_CHECK(hipMemcpyAsync(in_deriv->Data(), out_deriv.Data(),
                                    sizeof(float) * out_deriv.NumRows() * out_deriv.NumCols(),
                                    hipMemcpyDeviceToDevice, S()));
    return;
  }
  const long rows = out_deriv.NumRows();
  const int ns = (int)(in_deriv->NumRows() / rows);
  splice_rows_backward(S(), out_deriv.Data(), input_dim_, ns, rows, context_.data(), (int)context_.size(),
                       out_info.first_offset - in_info.first_offset, const_dim_, in_deriv->Data());
}
Component *SpliceComponent::Copy() const {
  auto *c = new SpliceComponent;
  c->input_dim_ = input_dim_;
  c->const_dim_ = const_dim_;
  c->context_ = context_;
  return c;
}
void SpliceComponent::Write(std::ostream &os, bool binary) const {  // :2822-2833
  WriteToken(os, binary, "<SpliceComponent>");
  WriteToken(os, binary, "<InputDim>");
  kio::WriteInt(os, binary, input_dim_);
  WriteToken(os, binary, "<Context>");
  kio::WriteIntVector(os, binary, std::vector<int32_t>(context_.begin(), context_.end()));
  WriteToken(os, binary, "<ConstComponentDim>");
  kio::WriteInt(os, binary, const_dim_);
  WriteToken(os, binary, "</SpliceComponent>");
}
// SpliceComponent::Read (nnet-component.cc:2797-2820), incl. the old
// <LeftContext>/<RightContext> form
void SpliceComponent::Read(std::istream &is, bool binary) {
  ExpectToken(is, binary, "<InputDim>");
  const int input_dim = kio::ReadInt(is, binary);
  const std::string t = kio::ReadToken(is, binary);
  std::vector<int> context;
  if (t == "<LeftContext>") {
    const int l = kio::ReadInt(is, binary);
    ExpectToken(is, binary, "<RightContext>");
    const int r = kio::ReadInt(is, binary);
    for (int i = -l; i <= r; i++) context.push_back(i);
  } else if (t == "<Context>") {
    for (int32_t c : kio::ReadIntVector(is, binary)) context.push_back(c);
  } else {
    throw std::runtime_error("SpliceComponent: unknown token " + t);
  }
  ExpectToken(is, binary, "<ConstComponentDim>");
  const int cdim = kio::ReadInt(is, binary);
  ExpectToken(is, binary, "</SpliceComponent>");
  if (input_dim <= 0) throw std::runtime_error("SpliceComponent: bad <InputDim>");
  Init(input_dim, context, cdim);
}
// ---------------------------------------------------------------------------
// CuDNNRecurrentComponent (nnet-cudnn-component.cc:56-772)
// ---------------------------------------------------------------------------
CuDNNRecurrentComponent::CuDNNRecurrentComponent() {
  desc_.mode = kLstm;
  desc_.dirs = 2;
  KCTC_HIP_CHECK(hipMalloc(&err_, 256));
  KCTC_HIP_CHECK(hipMemset(err_, 0, 256));
}
CuDNNRecurrentComponent::~CuDNNRecurrentComponent() {
  if (err_) (void)hipFree(err_);
  if (pre_.ev) (void)hipEventDestroy(pre_.ev);
  if (pre_.wev) (void)hipEventDestroy(pre_.wev);
}

void CuDNNRecurrentComponent::InitFromString(std::string args, Rng &rng) {
  const std::string orig = args;
  bool ok = true, bidir = true;
  int layers = 0, D = 0, H = 0, mode = 2, mb = 0;
  ok = ok && ParseFromString("learning-rate", &args, &learning_rate_);
  ok = ok && ParseFromString("num-layers", &args, &layers);
  ok = ok && ParseFromString("input-dim", &args, &D);
  ok = ok && ParseFromString("output-dim", &args, &H);
  ok = ok && ParseFromString("rnn-mode", &args, &mode);
  ok = ok && ParseFromString("bidirectional", &args, &bidir);
  ok = ok && ParseFromString("max-seq-length", &args, &max_seq_length_);
  ParseFromString("param-stddev", &args, &param_stddev_);
  ParseFromString("bias-stddev", &args, &bias_stddev_);
  ParseFromString("clip-gradient", &args, &clip_gradient_);
  ParseFromString("mini-batch", &args, &mb);
  if (!ok) throw std::invalid_argument("Bad initializer " + orig);
  if (mode < 0 || mode > 3)
    throw std::invalid_argument("rnn_mode_ = " + std::to_string(mode) + ", should in [0, 1, 2, 3].");
  desc_.mode = mode;
  desc_.D = D;
  desc_.H = H;
  desc_.layers = layers;
  desc_.dirs = bidir ? 2 : 1;
  Init(rng);
}

// weights: every lin-layer matrix ~ N(0, param_stddev^2), every bias vector =
// bias_stddev (SetRandn then Set, nnet-cudnn-component.cc:336-407)
void CuDNNRecurrentComponent::Init(Rng &rng) {
  const long P = desc_.params_size();
  std::vector<float> h((size_t)P, 0.f);
  const int nlin = 2 * desc_.nw();
  for (int pl = 0; pl < desc_.layers * desc_.dirs; pl++) {
    for (int lin = 0; lin < nlin; lin++) {
      const long off = desc_.lin_offset(pl, lin, false);
      const long n = (long)desc_.H * (lin < desc_.nw() ? desc_.din(pl / desc_.dirs) : desc_.H);
      for (long i = 0; i < n; i++) h[off + i] = (float)(rng.gauss() * param_stddev_);
      const long bo = desc_.lin_offset(pl, lin, true);
      for (long i = 0; i < desc_.H; i++) h[bo + i] = bias_stddev_;
    }
  }
  params_.ensure(sizeof(float) * P);
  grad_.ensure(sizeof(float) * P);
  h2d(params_.f(), h.data(), P);
}

std::string CuDNNRecurrentComponent::Info() const {
  std::ostringstream os;
  os << Type() << ", input-dim=" << desc_.D << ", output-dim=" << OutputDim()
     << ", learning-rate=" << learning_rate_ << ", hidden-dim=" << desc_.H
     << ", num-layers=" << desc_.layers << ", max-seq-length=" << max_seq_length_
     << ", rnn-mode=" << desc_.mode << (desc_.dirs == 2 ? ", BIDIRECTIONAL" : ", UNIDIRECTIONAL");
  return os.str();
}

void CuDNNRecurrentComponent::Propagate(const ChunkInfo &, const ChunkInfo &, const CuMatrixBase &in,
                                        CuMatrixBase *out) const {
  Forward(in, out, nullptr);
}

void CuDNNRecurrentComponent::PropagateChained(const CuMatrixBase &in, CuMatrixBase *out,
                                               const CuDNNRecurrentComponent &next) const {
  auto &dev = CuDevice::Instantiate();
  const int N = mini_batch_ > 0 ? mini_batch_ : 1;
  const int T = (int)(in.NumRows() / N);
  // |h| <= 1 for LSTM / GRU / TANH outputs: the next RNN's input needs no max pass
  next.input_bound_ = desc_.mode != kRelu ? 1.f : 0.f;
  if (!dev.side || next.mini_batch_ != N || next.desc_.D != OutputDim()) {
    Forward(in, out, nullptr);
    return;
  }
  next.reserve_.ensure(sizeof(float) * rnn_reserve_layout(next.desc_, T, N).total);
  next.workspace_.ensure(rnn_workspace_bytes(next.desc_, T, N));
  RnnFwdChain c;
  c.d = &next.desc_; c.w = next.params_.f();
  c.workspace = next.workspace_.p; c.ws_bytes = next.workspace_.bytes;
  c.reserve = next.reserve_.p; c.res_bytes = next.reserve_.bytes;
  c.side = dev.side;
  Forward(in, out, &c);
  next.input_projected_ = c.done;
}

void CuDNNRecurrentComponent::Forward(const CuMatrixBase &in, CuMatrixBase *out, RnnFwdChain *chain) const {
  // seq_length = rows / mini_batch, no masking (nnet-cudnn-component.cc:521-555)
  const int N = mini_batch_ > 0 ? mini_batch_ : 1;
  const int T = (int)(in.NumRows() / N);
  if (in.NumCols() != desc_.D || in.NumRows() % N)
    throw std::invalid_argument("CuDNNRecurrentComponent::Propagate: bad input shape");
  seq_length_ = T;
  reserve_.ensure(sizeof(float) * rnn_reserve_layout(desc_, T, N).total);
  workspace_.ensure(rnn_workspace_bytes(desc_, T, N));
  const bool projected = input_projected_;
  input_projected_ = false;
  in_tn_[0] = T;
  in_tn_[1] = N;
  ProfScope ps("layer_rnn_forward");
  // the trainer's side stream (idle during the forward pass): the W^T / x^T /
  // y^T prepacks beside the recurrence (rnn.h RnnPrepack)
  auto &dev = CuDevice::Instantiate();
  hipStream_t side = S() == dev.stream ? dev.side : nullptr;
  RnnPrepack *pre = nullptr;
  if ((prepack_dx_ || prepack_w_) && side) {
    if (!pre_.ev) KCTC_HIP_CHECK(hipEventCreateWithFlags(&pre_.ev, hipEventDisableTiming));
    if (!pre_.wev) KCTC_HIP_CHECK(hipEventCreateWithFlags(&pre_.wev, hipEventDisableTiming));
    // the dx-stream queue (idle in the forward pass): the side stream carries
    // the next component's projection streamed off this recurrence
    pre_.stream = dev.stream2 ? dev.stream2 : side;
    pre_.dx = prepack_dx_;
    pre_.wgrad = prepack_w_;
    pre_.in_bound = input_bound_;
    pre = &pre_;
  }
  pre_.done = pre_.wdone = false;
  pre_x_ = in.Data();
  pre_y_ = out->Data();
  int st = rnn_forward_training(desc_, S(), T, N, in.Data(), params_.f(), out->Data(), workspace_.p,
                                workspace_.bytes, reserve_.p, reserve_.bytes, DeviceError(), chain, projected, in_rows_,
                                pre);
  pre_ver_ = pver_;
  if (st) throw std::runtime_error("rnn_forward_training failed: " + std::to_string(st));
}

void CuDNNRecurrentComponent::Backprop(const ChunkInfo &, const ChunkInfo &,
                                       const CuMatrixBase &in_value, const CuMatrixBase &out_value,
                                       const CuMatrixBase &out_deriv, Component *to_update_in,
                                       CuMatrixBase *in_deriv) const {
  const int N = mini_batch_, T = seq_length_;
  auto &dev0 = CuDevice::Instantiate();
  // the bottom component (no input derivative): its weight gradients are
  // streamed off its own backward recurrence on the side stream (rnn.h
  // RnnWgradStream) instead of following it
  if (to_update_in && !in_deriv && dev0.side && rnn_wgrad_stream_ok(desc_, T, N)) {
    auto *to_update = dynamic_cast<CuDNNRecurrentComponent *>(to_update_in);
    if (!to_update) throw std::invalid_argument("CuDNNRecurrentComponent: bad to_update");
    hipStream_t ws = dev0.side;
    dev0.Fork();
    to_update->grad_stream_ = ws;
    KCTC_HIP_CHECK(hipMemsetAsync(to_update->grad_.p, 0, sizeof(float) * NumParameters(), ws));
    RnnWgradStream wg;
    wg.side = ws;
    if (const char *e = getenv("KCTC_WGRAD_CHUNKS")) wg.chunks = atoi(e);
    wg.x = in_value.Data();
    wg.dw = to_update->grad_.f();
    wg.max_blocks = side_gemm_blocks();
    wg.in_bound = input_bound_;
    {
      ProfScope ps("layer_rnn_backward_data");
      int st = rnn_backward_data(desc_, S(), T, N, out_value.Data(), out_deriv.Data(), params_.f(), nullptr,
                                 workspace_.p, workspace_.bytes, reserve_.p, reserve_.bytes, DeviceError(),
                                 dev0.stream2, &wg);
      if (st) throw std::runtime_error("rnn_backward_data failed: " + std::to_string(st));
    }
    if (!wg.done) {
      dev0.Fork();
      ProfScope ps("layer_rnn_backward_weights", ws);
      int st = rnn_backward_weights(desc_, ws, T, N, in_value.Data(), out_value.Data(), workspace_.p,
                                    workspace_.bytes, to_update->grad_.f(), reserve_.p, reserve_.bytes,
                                    side_gemm_blocks(), input_bound_, nullptr, packed_input_cols(T, N), false,
                                    wgrad_prepack(in_value, out_value));
      if (st) throw std::runtime_error("rnn_backward_weights failed: " + std::to_string(st));
    }
    return;
  }
  {
    ProfScope ps("layer_rnn_backward_data");
    // the forward's packed W^T, if the parameters are still the ones it packed
    const RnnPrepack *pre = pre_.done && pre_ver_ == pver_ ? &pre_ : nullptr;
    int st = rnn_backward_data(desc_, S(), T, N, out_value.Data(), out_deriv.Data(), params_.f(),
                               in_deriv ? in_deriv->Data() : nullptr, workspace_.p, workspace_.bytes,
                               reserve_.p, reserve_.bytes, DeviceError(), CuDevice::Instantiate().stream2, nullptr,
                               pre);
    if (st) throw std::runtime_error("rnn_backward_data failed: " + std::to_string(st));
  }
  if (to_update_in) {
    auto *to_update = dynamic_cast<CuDNNRecurrentComponent *>(to_update_in);
    if (!to_update) throw std::invalid_argument("CuDNNRecurrentComponent: bad to_update");
    // filter_params_grad_ is zeroed, then cudnnRNNBackwardWeights accumulates.
    // On the side stream (when there is one) so the weight GEMMs overlap the
    // next component's backward recurrence; only this component's reserve,
    // workspace and gradient are touched there.
    auto &dev = CuDevice::Instantiate();
    hipStream_t ws = dev.side ? dev.side : S();
    dev.Fork();
    to_update->grad_stream_ = ws;
    KCTC_HIP_CHECK(hipMemsetAsync(to_update->grad_.p, 0, sizeof(float) * NumParameters(), ws));
    ProfScope ps("layer_rnn_backward_weights", ws);
    // the bottom component (no input derivative): its weight GEMMs are the
    // step's tail, so dW runs beside dR on the (then idle) dx-stream queue
    int st = rnn_backward_weights(desc_, ws, T, N, in_value.Data(), out_value.Data(), workspace_.p,
                                  workspace_.bytes, to_update->grad_.f(), reserve_.p, reserve_.bytes,
                                  dev.side ? side_gemm_blocks() : 0, input_bound_,
                                  (!in_deriv && dev.side) ? dev.stream2 : nullptr, packed_input_cols(T, N),
                                  in_deriv && dev.side,  // the next component's backward runs beside
                                  wgrad_prepack(in_value, out_value));
    if (st) throw std::runtime_error("rnn_backward_weights failed: " + std::to_string(st));
  }
}

// x^T / y^T packed by the last forward, if this backward is for that forward's data
const RnnPrepack *CuDNNRecurrentComponent::wgrad_prepack(const CuMatrixBase &in_value,
                                                         const CuMatrixBase &out_value) const {
  return pre_.wdone && in_value.Data() == pre_x_ && out_value.Data() == pre_y_ ? &pre_ : nullptr;
}

bool CuDNNRecurrentComponent::PackedOutput(const void **rows, const void **cols) const {
  *rows = *cols = nullptr;
  if (!reserve_.p || seq_length_ <= 0 || mini_batch_ <= 0) return false;
  if (reserve_.bytes < sizeof(float) * (size_t)rnn_reserve_layout(desc_, seq_length_, mini_batch_).total) return false;
  return rnn_packed_output(desc_, seq_length_, mini_batch_, reserve_.p, rows, cols);
}

hipStream_t UpdatableComponent::GradStream() const { return grad_stream_ ? grad_stream_ : S(); }

void UpdatableComponent::SetMomentum(float m) {
  if (!(m >= 0.f && m < 1.f)) throw std::invalid_argument("momentum must be in [0, 1)");
  momentum_ = m;
  if (m != 0.f) {  // delta_nnet->SetZero(false): a fresh zero delta
    delta_.ensure(sizeof(float) * NumParameters());
    KCTC_HIP_CHECK(hipMemsetAsync(delta_.p, 0, sizeof(float) * NumParameters(), S()));
  }
}

void UpdatableComponent::UpdateWith(float *params, const float *grad, float clip, const unsigned *skip) {
  if (momentum_ == 0.f)
    clip_sgd_update(S(), params, grad, NumParameters(), learning_rate_, clip, skip);
  else
    momentum_update(S(), params, delta_.f(), grad, NumParameters(), learning_rate_, clip, momentum_, skip);
}

// ---- UpdatableComponent parameter arithmetic (nnet-component.h:295-318) ----
static unsigned long long g_perturb_seed = 20161015ull, g_perturb_calls = 0;
void UpdatableComponent::SetPerturbSeed(unsigned long long seed) {
  g_perturb_seed = seed;
  g_perturb_calls = 0;
}

void UpdatableComponent::CopyUpdatableFrom(const UpdatableComponent &o) {
  learning_rate_ = o.learning_rate_;
  is_gradient_ = o.is_gradient_;
}

void UpdatableComponent::CheckSameKind(const UpdatableComponent &o, const char *what) const {
  if (o.Type() != Type() || o.NumParameters() != NumParameters())
    throw std::invalid_argument(std::string(what) + ": components of different type or size (" + Type() + " vs " +
                                o.Type() + ")");
}

void UpdatableComponent::SetZero(bool treat_as_gradient) {
  if (treat_as_gradient) {
    SetLearningRate(1.0f);
    is_gradient_ = true;
  }
  KCTC_HIP_CHECK(hipMemsetAsync(ParamData(), 0, sizeof(float) * NumParameters(), S()));
}

double UpdatableComponent::DotProduct(const UpdatableComponent &other) const {
  CheckSameKind(other, "DotProduct");
  auto *self = const_cast<UpdatableComponent *>(this);
  auto *o = const_cast<UpdatableComponent *>(&other);
  DevBuf ws;
  ws.ensure(dot_ws_bytes() + sizeof(double));
  double *out = reinterpret_cast<double *>(static_cast<char *>(ws.p) + dot_ws_bytes());
  // the other component's parameters may still be written on its own stream
  KCTC_HIP_CHECK(hipStreamSynchronize(o->GradStream()));
  dot_f64(S(), self->ParamData(), o->ParamData(), NumParameters(), out, ws.p);
  double h = 0;
  KCTC_HIP_CHECK(hipMemcpyAsync(&h, out, sizeof(double), hipMemcpyDeviceToHost, S()));
  KCTC_HIP_CHECK(hipStreamSynchronize(S()));
  return h;
}

void UpdatableComponent::PerturbParams(float stddev) {
  Rng r(g_perturb_seed + 0x51ED27ull * ++g_perturb_calls);
  add_randn(S(), ParamData(), NumParameters(), stddev, r.next());
}

void UpdatableComponent::Scale(float scale) { scale_inplace(S(), ParamData(), NumParameters(), scale); }

void UpdatableComponent::Add(float alpha, const UpdatableComponent &other) {
  CheckSameKind(other, "Add");
  axpy(S(), ParamData(), const_cast<UpdatableComponent &>(other).ParamData(), NumParameters(), alpha);
}

int CuDNNRecurrentComponent::side_gemm_blocks() const {
  return 512;  // dynamic tile scheduling: two per CU, late starters exit
}

void CuDNNRecurrentComponent::ApplyUpdate(const unsigned *skip) {
  // ApplyFloor(-clip) / ApplyCeiling(clip) then filter_params_ += lr * grad
  ++pver_;
  UpdateWith(params_.f(), grad_.f(), clip_gradient_, skip);
}

// CuDNNRecurrentComponent(const CuDNNRecurrentComponent &) (nnet-cudnn-component.cc:650-671):
// configuration and filter_params_, no minibatch state (mini_batch_ = 0)
Component *CuDNNRecurrentComponent::Copy() const {
  auto *c = new CuDNNRecurrentComponent;
  c->CopyUpdatableFrom(*this);
  c->desc_ = desc_;
  c->max_seq_length_ = max_seq_length_;
  c->param_stddev_ = param_stddev_;
  c->bias_stddev_ = bias_stddev_;
  c->clip_gradient_ = clip_gradient_;
  const long P = NumParameters();
  c->params_.ensure(sizeof(float) * P);
  c->grad_.ensure(sizeof(float) * P);
  KCTC_HIP_CHECK(hipMemcpyAsync(c->params_.p, params_.p, sizeof(float) * P, hipMemcpyDeviceToDevice, S()));
  return c;
}

// :723-730 (SetBufferZero: the reserve is rebuilt by the next Propagate here)
void CuDNNRecurrentComponent::SetZero(bool treat_as_gradient) {
  UpdatableComponent::SetZero(treat_as_gradient);
  input_projected_ = false;
}

void CuDNNRecurrentComponent::Vectorize(float *host) const {
  auto v = d2h(params_.f(), NumParameters());
  std::copy(v.begin(), v.end(), host);
}
void CuDNNRecurrentComponent::UnVectorize(const float *host) {
  ++pver_;
  h2d(params_.f(), host, NumParameters());
}

// nnet-cudnn-component.cc:698-721
void CuDNNRecurrentComponent::Write(std::ostream &os, bool binary) const {
  WriteToken(os, binary, "<CuDNNRecurrentComponent>");
  WriteToken(os, binary, "<LearningRate>");
  kio::WriteFloat(os, binary, learning_rate_);
  WriteToken(os, binary, "<IsGradient>");
  kio::WriteBool(os, binary, is_gradient_);
  WriteToken(os, binary, "<ClipGradient>");
  kio::WriteFloat(os, binary, clip_gradient_);
  WriteToken(os, binary, "<InputDim>");
  kio::WriteInt(os, binary, desc_.D);
  WriteToken(os, binary, "<HiddenDim>");
  kio::WriteInt(os, binary, desc_.H);
  WriteToken(os, binary, "<NumLayers>");
  kio::WriteInt(os, binary, desc_.layers);
  WriteToken(os, binary, "<Bidirectional>");
  kio::WriteBool(os, binary, desc_.dirs == 2);
  WriteToken(os, binary, "<RNNMode>");
  kio::WriteInt(os, binary, desc_.mode);
  WriteToken(os, binary, "<MaxSeqLength>");
  kio::WriteInt(os, binary, max_seq_length_);
  WriteToken(os, binary, "<FilterParams>");
  auto v = d2h(params_.f(), NumParameters());
  kio::WriteFloatVector(os, binary, v.data(), (long)v.size());
  WriteToken(os, binary, "</CuDNNRecurrentComponent>");
}// nnet-cudnn-component.cc:673-696
void CuDNNRecurrentComponent::Read(std::istream &is, bool binary) {
  ExpectToken(is, binary, "<LearningRate>");
  learning_rate_ = kio::ReadFloat(is, binary);
  ExpectToken(is, binary, "<IsGradient>");
  is_gradient_ = kio::ReadBool(is, binary);
  ExpectToken(is, binary, "<ClipGradient>");
  clip_gradient_ = kio::ReadFloat(is, binary);
  ExpectToken(is, binary, "<InputDim>");
  desc_.D = kio::ReadInt(is, binary);
  ExpectToken(is, binary, "<HiddenDim>");
  desc_.H = kio::ReadInt(is, binary);
  ExpectToken(is, binary, "<NumLayers>");
  desc_.layers = kio::ReadInt(is, binary);
  ExpectToken(is, binary, "<Bidirectional>");
  desc_.dirs = kio::ReadBool(is, binary) ? 2 : 1;
  ExpectToken(is, binary, "<RNNMode>");
  desc_.mode = kio::ReadInt(is, binary);
  ExpectToken(is, binary, "<MaxSeqLength>");
  max_seq_length_ = kio::ReadInt(is, binary);
  // InitFromString's checks (nnet-cudnn-component.cc:72-98), before any size is trusted
  if (desc_.mode < 0 || desc_.mode > 3)
    throw std::runtime_error("CuDNNRecurrentComponent: rnn_mode_ = " + std::to_string(desc_.mode) +
                             ", should in [0, 1, 2, 3].");
  if (desc_.D <= 0 || desc_.H <= 0 || desc_.layers <= 0 || max_seq_length_ <= 0)
    throw std::runtime_error("CuDNNRecurrentComponent: bad dimensions in model file");
  ExpectToken(is, binary, "<FilterParams>");
  auto v = kio::ReadFloatVector(is, binary);
  if ((long)v.size() != desc_.params_size())
    throw std::runtime_error("CuDNNRecurrentComponent: FilterParams size mismatch");
  params_.ensure(sizeof(float) * v.size());
  grad_.ensure(sizeof(float) * v.size());
  h2d(params_.f(), v.data(), (long)v.size());
  ExpectToken(is, binary, "</CuDNNRecurrentComponent>");
}
// ---------------------------------------------------------------------------
// ClipGradientComponent (nnet-cudnn-component.cc:775-1075)
// ---------------------------------------------------------------------------
ClipGradientComponent::ClipGradientComponent() {
  KCTC_HIP_CHECK(hipMalloc(&dev_, sizeof(ClipState)));
  KCTC_HIP_CHECK(hipMemset(dev_, 0, sizeof(ClipState)));
}
ClipGradientComponent::~ClipGradientComponent() {
  delete shadow_;
  if (dev_) (void)hipFree(dev_);
}

// delta_nnet = new Nnet(*nnet): the copy starts with this component's
// configuration and counters (ctc-nnet-train.cc:194-202)
void ClipGradientComponent::EnableShadow(bool on) {
  delete shadow_;
  shadow_ = nullptr;
  if (!on) return;
  auto *c = new ClipGradientComponent();
  c->dim_ = dim_;
  c->clipping_threshold_ = clipping_threshold_;
  c->norm_based_clipping_ = norm_based_clipping_;
  c->self_repair_clipped_proportion_threshold_ = self_repair_clipped_proportion_threshold_;
  c->self_repair_target_ = self_repair_target_;
  c->self_repair_scale_ = self_repair_scale_;
  SyncStats();
  c->num_clipped_ = num_clipped_;
  c->count_ = count_;
  c->num_self_repaired_ = num_self_repaired_;
  c->num_backpropped_ = num_backpropped_;
  KCTC_HIP_CHECK(hipMemcpyAsync(c->dev_, dev_, sizeof(ClipState), hipMemcpyDeviceToDevice, S()));
  shadow_ = c;
}

void ClipGradientComponent::InitFromString(std::string args, Rng &) {
  const std::string orig = args;
  bool ok = ParseFromString("dim", &args, &dim_);
  clipping_threshold_ = 15.0f;
  norm_based_clipping_ = false;
  self_repair_clipped_proportion_threshold_ = 0.01f;
  self_repair_target_ = 0.0f;
  self_repair_scale_ = 1.0f;
  ParseFromString("clipping-threshold", &args, &clipping_threshold_);
  ParseFromString("norm-based-clipping", &args, &norm_based_clipping_);
  ParseFromString("self-repair-clipped-proportion-threshold", &args,
                  &self_repair_clipped_proportion_threshold_);
  ParseFromString("self-repair-target", &args, &self_repair_target_);
  ParseFromString("self-repair-scale", &args, &self_repair_scale_);
  if (!ok || !args.empty() || clipping_threshold_ < 0 || dim_ <= 0 ||
      self_repair_clipped_proportion_threshold_ < 0 || self_repair_target_ < 0 ||
      self_repair_scale_ < 0)
    throw std::invalid_argument("Invalid initializer for layer of type ClipGradientComponent: \"" +
                                orig + "\"");
  ZeroStats();
}

std::string ClipGradientComponent::Info() const {
  SyncStats();
  std::ostringstream os;
  os << Type() << ", dim=" << dim_ << ", norm-based-clipping=" << (norm_based_clipping_ ? "true" : "false")
     << ", clipping-threshold=" << clipping_threshold_
     << ", clipped-proportion=" << (count_ > 0 ? num_clipped_ / count_ : 0.0);
  if (self_repair_scale_ != 0.0f)
    os << ", self-repair-clipped-proportion-threshold=" << self_repair_clipped_proportion_threshold_
       << ", self-repair-target=" << self_repair_target_ << ", self-repair-scale=" << self_repair_scale_;
  return os.str();
}

void ClipGradientComponent::Propagate(const ChunkInfo &, const ChunkInfo &, const CuMatrixBase &in,
                                      CuMatrixBase *out) const {
  if (out->Data() != in.Data())
    KCTC_HIP_CHECK(hipMemcpyAsync(out->Data(), in.Data(), sizeof(float) * in.NumRows() * in.NumCols(),
                                  hipMemcpyDeviceToDevice, S()));
}

void ClipGradientComponent::Backprop(const ChunkInfo &, const ChunkInfo &, const CuMatrixBase &in_value,
                                     const CuMatrixBase &, const CuMatrixBase &out_deriv,
                                     Component *to_update_in, CuMatrixBase *in_deriv) const {
  if (!in_deriv) return;
  if (in_deriv->Data() != out_deriv.Data())
    KCTC_HIP_CHECK(hipMemcpyAsync(in_deriv->Data(), out_deriv.Data(),
                                  sizeof(float) * out_deriv.NumRows() * out_deriv.NumCols(),
                                  hipMemcpyDeviceToDevice, S()));
  auto *to_update = dynamic_cast<ClipGradientComponent *>(to_update_in);
  if (!(clipping_threshold_ > 0)) return;
  const long rows = in_deriv->NumRows();
  // RepairGradients' host-side gate, in the reference's short-circuit order
  // (:988-991): the RandUniform() draw is consumed only when the preceding
  // conditions pass.  count_ includes this minibatch when norm-based.
  bool try_repair = false;
  if (to_update) {
    to_update->num_backpropped_ += 1;
    const double count_after = count_ + ((norm_based_clipping_ && to_update == this) ? rows : 0);
    if (!(self_repair_clipped_proportion_threshold_ >= 1.0f || self_repair_scale_ == 0.0f ||
          count_after == 0)) {
      if (!rng_) throw std::logic_error("ClipGradientComponent: no random stream for self-repair");
      try_repair = !(rng_->RandUniform() > 0.5f);  // RandUniform() > repair_probability
    }
    if (norm_based_clipping_) to_update->count_ += rows;
  }
  ProfScope ps("clip_gradient");
  scratch_.ensure(clipgrad_scratch_bytes(rows));
  clipgrad_backprop(S(), in_deriv->Data(), in_value.Data(), rows, dim_, clipping_threshold_,
                    norm_based_clipping_, try_repair, self_repair_clipped_proportion_threshold_,
                    self_repair_target_, self_repair_scale_, (to_update ? to_update : this)->dev_,
                    scratch_.p, dev_);
}

Component *ClipGradientComponent::Copy() const {
  auto *c = new ClipGradientComponent;
  c->dim_ = dim_;
  c->clipping_threshold_ = clipping_threshold_;
  c->norm_based_clipping_ = norm_based_clipping_;
  c->self_repair_clipped_proportion_threshold_ = self_repair_clipped_proportion_threshold_;
  c->self_repair_target_ = self_repair_target_;
  c->self_repair_scale_ = self_repair_scale_;
  SyncStats();
  c->num_clipped_ = num_clipped_;
  c->count_ = count_;
  c->num_self_repaired_ = num_self_repaired_;
  c->num_backpropped_ = num_backpropped_;
  KCTC_HIP_CHECK(hipMemcpyAsync(c->dev_, dev_, sizeof(ClipState), hipMemcpyDeviceToDevice, S()));
  return c;
}

// the device counters are the truth during training; scaled on the host and
// written back (both are off the per-step path)
void ClipGradientComponent::Scale(float scale) {  // :1064-1067
  SyncStats();
  count_ *= scale;
  num_clipped_ *= scale;
  ClipState h{};
  h.num_clipped = num_clipped_;
  h.count = count_;
  h.num_self_repaired = num_self_repaired_;
  KCTC_HIP_CHECK(hipMemcpyAsync(dev_, &h, sizeof(h), hipMemcpyHostToDevice, S()));
  KCTC_HIP_CHECK(hipStreamSynchronize(S()));
}

void ClipGradientComponent::Add(float alpha, const ClipGradientComponent &other) {  // :1069-1073
  SyncStats();
  other.SyncStats();
  count_ += alpha * other.count_;
  num_clipped_ += alpha * other.num_clipped_;
  ClipState h{};
  h.num_clipped = num_clipped_;
  h.count = count_;
  h.num_self_repaired = num_self_repaired_;
  KCTC_HIP_CHECK(hipMemcpyAsync(dev_, &h, sizeof(h), hipMemcpyHostToDevice, S()));
  KCTC_HIP_CHECK(hipStreamSynchronize(S()));
}

void ClipGradientComponent::SyncStats() const {
  ClipState h;
  KCTC_HIP_CHECK(hipMemcpyAsync(&h, dev_, sizeof(h), hipMemcpyDeviceToHost, S()));
  KCTC_HIP_CHECK(hipStreamSynchronize(S()));
  num_clipped_ = h.num_clipped;
  count_ = h.count;
  num_self_repaired_ = h.num_self_repaired;
}

void ClipGradientComponent::ZeroStats() {
  KCTC_HIP_CHECK(hipMemsetAsync(dev_, 0, sizeof(ClipState), S()));
  num_clipped_ = count_ = num_self_repaired_ = num_backpropped_ = 0;
}

// nnet-cudnn-component.cc:814-837
void ClipGradientComponent::Write(std::ostream &os, bool binary) const {
  SyncStats();
  WriteToken(os, binary, "<ClipGradientComponent>");
  WriteToken(os, binary, "<Dim>");
  kio::WriteInt(os, binary, dim_);
  WriteToken(os, binary, "<ClippingThreshold>");
  kio::WriteFloat(os, binary, clipping_threshold_);
  WriteToken(os, binary, "<NormBasedClipping>");
  kio::WriteBool(os, binary, norm_based_clipping_);
  WriteToken(os, binary, "<SelfRepairClippedProportionThreshold>");
  kio::WriteFloat(os, binary, self_repair_clipped_proportion_threshold_);
  WriteToken(os, binary, "<SelfRepairTarget>");
  kio::WriteFloat(os, binary, self_repair_target_);
  WriteToken(os, binary, "<SelfRepairScale>");
  kio::WriteFloat(os, binary, self_repair_scale_);
  WriteToken(os, binary, "<NumElementsClipped>");
  kio::WriteInt(os, binary, as_i32(num_clipped_));
  WriteToken(os, binary, "<NumElementsProcessed>");
  kio::WriteInt(os, binary, as_i32(count_));
  WriteToken(os, binary, "<NumSelfRepaired>");
  kio::WriteInt(os, binary, as_i32(num_self_repaired_));
  WriteToken(os, binary, "<NumBackpropped>");
  kio::WriteInt(os, binary, as_i32(num_backpropped_));
  WriteToken(os, binary, "</ClipGradientComponent>");
}// nnet-cudnn-component.cc:775-812 (older files without the self-repair fields)
void ClipGradientComponent::Read(std::istream &is, bool binary) {
  ExpectToken(is, binary, "<Dim>");
  dim_ = kio::ReadInt(is, binary);
  ExpectToken(is, binary, "<ClippingThreshold>");
  clipping_threshold_ = kio::ReadFloat(is, binary);
  ExpectToken(is, binary, "<NormBasedClipping>");
  norm_based_clipping_ = kio::ReadBool(is, binary);
  std::string t = kio::ReadToken(is, binary);
  if (t == "<SelfRepairClippedProportionThreshold>") {
    self_repair_clipped_proportion_threshold_ = kio::ReadFloat(is, binary);
    ExpectToken(is, binary, "<SelfRepairTarget>");
    self_repair_target_ = kio::ReadFloat(is, binary);
    ExpectToken(is, binary, "<SelfRepairScale>");
    self_repair_scale_ = kio::ReadFloat(is, binary);
    ExpectToken(is, binary, "<NumElementsClipped>");
  } else {
    self_repair_clipped_proportion_threshold_ = 1.0f;
    self_repair_target_ = 0.0f;
    self_repair_scale_ = 0.0f;
    if (t != "<NumElementsClipped>") throw std::runtime_error("ClipGradientComponent: bad token " + t);
  }
  num_clipped_ = kio::ReadInt(is, binary);
  ExpectToken(is, binary, "<NumElementsProcessed>");
  count_ = kio::ReadInt(is, binary);
  t = kio::ReadToken(is, binary);
  if (t == "<NumSelfRepaired>") {
    num_self_repaired_ = kio::ReadInt(is, binary);
    ExpectToken(is, binary, "<NumBackpropped>");
    num_backpropped_ = kio::ReadInt(is, binary);
    ExpectToken(is, binary, "</ClipGradientComponent>");
  } else {
    num_self_repaired_ = num_backpropped_ = 0;
    if (t != "</ClipGradientComponent>") throw std::runtime_error("ClipGradientComponent: bad token " + t);
  }
  ClipState h{};
  h.num_clipped = num_clipped_;
  h.count = count_;
  h.num_self_repaired = num_self_repaired_;
  KCTC_HIP_CHECK(hipMemcpy(dev_, &h, sizeof(h), hipMemcpyHostToDevice));
}
// ---------------------------------------------------------------------------
// SoftmaxComponent (NonlinearComponent I/O, nnet-component.cc:383-426)
// ---------------------------------------------------------------------------
void SoftmaxComponent::InitFromString(std::string args, Rng &) {
  const std::string orig = args;
  const bool ok = ParseFromString("dim", &args, &dim_);
  if (!ok || !args.empty() || dim_ <= 0)
    throw std::invalid_argument("Invalid initializer for layer of type SoftmaxComponent: \"" + orig + "\"");
  value_sum_.clear();
  deriv_sum_.clear();
  count_ = 0;
}
void SoftmaxComponent::Propagate(const ChunkInfo &, const ChunkInfo &, const CuMatrixBase &in,
                                 CuMatrixBase *out) const {
  ProfScope ps("softmax");
  softmax_rows(S(), in.Data(), in.NumRows(), dim_, out->Data());  // ApplySoftMaxPerRow + ApplyFloor(1e-20)
}
void SoftmaxComponent::Backprop(const ChunkInfo &, const ChunkInfo &, const CuMatrixBase &,
                                const CuMatrixBase &out_value, const CuMatrixBase &out_deriv, Component *to_update_in,
                                CuMatrixBase *in_deriv) const {
  const long rows = out_deriv.NumRows();
  if (in_deriv) diff_softmax_rows(S(), out_value.Data(), out_deriv.Data(), rows, dim_, in_deriv->Data());
  if (to_update_in) {  // NonlinearComponent::UpdateStats(out_value) (:337-363): value_sum_ += column sums, count_ += rows
    auto *to_update = dynamic_cast<SoftmaxComponent *>(to_update_in);
    if (!to_update) throw std::invalid_argument("SoftmaxComponent: bad to_update");
    ws_.ensure(sizeof(float) * ((size_t)dim_ + sum_rows_ws_floats(rows, dim_)));
    sum_rows(S(), out_value.Data(), rows, dim_, 1.f, 0.f, ws_.f(), ws_.f() + dim_);
    auto v = d2h(ws_.f(), dim_);
    if (to_update->value_sum_.empty()) to_update->value_sum_.assign(dim_, 0.0);
    for (int j = 0; j < dim_; j++) to_update->value_sum_[j] += v[j];
    to_update->count_ += (double)rows;
  }
}
Component *SoftmaxComponent::Copy() const {
  auto *c = new SoftmaxComponent;
  c->dim_ = dim_;
  c->value_sum_ = value_sum_;
  c->deriv_sum_ = deriv_sum_;
  c->count_ = count_;
  return c;
}
void SoftmaxComponent::Scale(float scale) {  // NonlinearComponent::Scale (nnet-component.cc:365-369)
  for (auto &v : value_sum_) v *= scale;
  for (auto &v : deriv_sum_) v *= scale;
  count_ *= scale;
}
void SoftmaxComponent::Add(float alpha, const SoftmaxComponent &other) {  // NonlinearComponent::Add (:371-382)
  if (value_sum_.empty() && !other.value_sum_.empty()) value_sum_.assign(other.value_sum_.size(), 0.0);
  if (deriv_sum_.empty() && !other.deriv_sum_.empty()) deriv_sum_.assign(other.deriv_sum_.size(), 0.0);
  for (size_t j = 0; j < other.value_sum_.size() && j < value_sum_.size(); j++) value_sum_[j] += alpha * other.value_sum_[j];
  for (size_t j = 0; j < other.deriv_sum_.size() && j < deriv_sum_.size(); j++) deriv_sum_[j] += alpha * other.deriv_sum_[j];
  count_ += alpha * other.count_;
}
void SoftmaxComponent::Write(std::ostream &os, bool binary) const {
  WriteToken(os, binary, "<SoftmaxComponent>");
  WriteToken(os, binary, "<Dim>");
  kio::WriteInt(os, binary, dim_);
  WriteToken(os, binary, "<ValueSum>");
  kio::WriteDoubleVector(os, binary, value_sum_);
  WriteToken(os, binary, "<DerivSum>");
  kio::WriteDoubleVector(os, binary, deriv_sum_);
  WriteToken(os, binary, "<Count>");
  kio::WriteDouble(os, binary, count_);
  WriteToken(os, binary, "</SoftmaxComponent>");
}
void SoftmaxComponent::Read(std::istream &is, bool binary) {
  // ExpectOneOrTwoTokens(<SoftmaxComponent>, <Dim>): the type token was consumed by Nnet::Read
  ExpectToken(is, binary, "<Dim>");
  dim_ = kio::ReadInt(is, binary);
  if (dim_ <= 0) throw std::runtime_error("SoftmaxComponent: bad <Dim>");
  ExpectToken(is, binary, "<ValueSum>");
  value_sum_ = kio::ReadDoubleVector(is, binary);
  ExpectToken(is, binary, "<DerivSum>");
  deriv_sum_ = kio::ReadDoubleVector(is, binary);
  ExpectToken(is, binary, "<Count>");
  count_ = kio::ReadDouble(is, binary);
  ExpectToken(is, binary, "</SoftmaxComponent>");
}
// ---------------------------------------------------------------------------
// AffineComponent (nnet-component.cc:1125-1274)
// ---------------------------------------------------------------------------
void AffineComponent::InitFromString(std::string args, Rng &rng) {
  const std::string orig = args;
  bool ok = true;
  ParseFromString("learning-rate", &args, &learning_rate_);
  ok = ok && ParseFromString("input-dim", &args, &in_dim_);
  ok = ok && ParseFromString("output-dim", &args, &out_dim_);
  if (!ok || in_dim_ <= 0 || out_dim_ <= 0) throw std::invalid_argument("Bad initializer " + orig);
  float param_stddev = 1.0f / std::sqrt((float)in_dim_), bias_stddev = 1.0f;
  ParseFromString("param-stddev", &args, &param_stddev);
  ParseFromString("bias-stddev", &args, &bias_stddev);
  if (!args.empty()) throw std::invalid_argument("Could not process these elements in initializer: " + args);
  std::vector<float> h((size_t)NumParameters());
  for (long i = 0; i < (long)in_dim_ * out_dim_; i++) h[i] = (float)(rng.gauss() * param_stddev);
  for (int i = 0; i < out_dim_; i++) h[(long)in_dim_ * out_dim_ + i] = (float)(rng.gauss() * bias_stddev);
  params_.ensure(sizeof(float) * h.size());
  grad_.ensure(sizeof(float) * h.size());
  h2d(params_.f(), h.data(), (long)h.size());
}

std::string AffineComponent::Info() const {
  std::ostringstream os;
  os << Type() << ", input-dim=" << in_dim_ << ", output-dim=" << out_dim_
     << ", learning-rate=" << learning_rate_;
  return os.str();
}

void AffineComponent::Propagate(const ChunkInfo &, const ChunkInfo &, const CuMatrixBase &in,
                                CuMatrixBase *out) const {
  // out = 1 b^T + in W^T (CopyRowsFromVec + AddMatMat, :1184-1196), fused bias
  ProfScope ps("affine");
  GemmArgs g;
  g.transA = false; g.transB = true;
  g.M = (int)in.NumRows(); g.N = out_dim_; g.K = in_dim_;
  g.A = in.Data(); g.lda = in_dim_;
  g.B = params_.f(); g.ldb = in_dim_;
  g.C = out->Data(); g.ldc = out_dim_;
  g.bias = params_.f() + (long)in_dim_ * out_dim_;
  gemm_f32(S(), g);
}

void AffineComponent::Backprop(const ChunkInfo &, const ChunkInfo &, const CuMatrixBase &in_value,
                               const CuMatrixBase &, const CuMatrixBase &out_deriv,
                               Component *to_update_in, CuMatrixBase *in_deriv) const {
  ProfScope ps("affine");
  const long rows = out_deriv.NumRows();
  if (in_deriv) {  // in_deriv = out_deriv W
    GemmArgs g;
    g.M = (int)rows; g.N = in_dim_; g.K = out_dim_;
    g.A = out_deriv.Data(); g.lda = out_dim_;
    g.B = params_.f(); g.ldb = in_dim_;
    g.C = in_deriv->Data(); g.ldc = in_dim_;
    gemm_f32(S(), g);
  }
  if (to_update_in) {
    auto *to_update = dynamic_cast<AffineComponent *>(to_update_in);
    if (!to_update) throw std::invalid_argument("AffineComponent: bad to_update");
    // UpdateSimple (:1190-1195): grad_W = out_deriv^T in_value, grad_b = row sum
    GemmArgs g;
    g.transA = true;
    g.M = out_dim_; g.N = in_dim_; g.K = (int)rows;
    g.A = out_deriv.Data(); g.lda = out_dim_;
    g.B = in_value.Data(); g.ldb = in_dim_;
    g.C = to_update->grad_.f(); g.ldc = in_dim_;
    g.split_k = gemm_pick_split(g.M, g.N, g.K, 1);
    const size_t wsf = (size_t)g.split_k * g.M * g.N + sum_rows_ws_floats(rows, out_dim_);
    ws_.ensure(sizeof(float) * wsf);
    g.ws = ws_.f();
    gemm_f32(S(), g);
    sum_rows(S(), out_deriv.Data(), rows, out_dim_, 1.f, 0.f,
             to_update->grad_.f() + (long)in_dim_ * out_dim_, ws_.f() + (size_t)g.split_k * g.M * g.N);
  }
}

Component *AffineComponent::Copy() const {  // AffineComponent(const AffineComponent &) (:1046-1050)
  auto *c = new AffineComponent;
  c->CopyUpdatableFrom(*this);
  c->in_dim_ = in_dim_;
  c->out_dim_ = out_dim_;
  const long P = NumParameters();
  c->params_.ensure(sizeof(float) * P);
  c->grad_.ensure(sizeof(float) * P);
  KCTC_HIP_CHECK(hipMemcpyAsync(c->params_.p, params_.p, sizeof(float) * P, hipMemcpyDeviceToDevice, S()));
  return c;
}

void AffineComponent::ApplyUpdate(const unsigned *skip) {
  UpdateWith(params_.f(), grad_.f(), 0.f, skip);
}
void AffineComponent::Vectorize(float *host) const {
  auto v = d2h(params_.f(), NumParameters());
  std::copy(v.begin(), v.end(), host);
}
void AffineComponent::UnVectorize(const float *host) { h2d(params_.f(), host, NumParameters()); }

// nnet-component.cc:1260-1274
void AffineComponent::Write(std::ostream &os, bool binary) const {
  auto v = d2h(params_.f(), NumParameters());
  WriteToken(os, binary, "<AffineComponent>");
  WriteToken(os, binary, "<LearningRate>");
  kio::WriteFloat(os, binary, learning_rate_);
  WriteToken(os, binary, "<LinearParams>");
  kio::WriteFloatMatrix(os, binary, v.data(), out_dim_, in_dim_);
  WriteToken(os, binary, "<BiasParams>");
  kio::WriteFloatVector(os, binary, v.data() + (long)in_dim_ * out_dim_, out_dim_);
  WriteToken(os, binary, "<IsGradient>");
  kio::WriteBool(os, binary, is_gradient_);
  WriteToken(os, binary, "</AffineComponent>");
}// nnet-component.cc:1228-1258 (incl. the <AvgInput> back-compatibility fields)
void AffineComponent::Read(std::istream &is, bool binary) {
  ExpectToken(is, binary, "<LearningRate>");
  learning_rate_ = kio::ReadFloat(is, binary);
  ExpectToken(is, binary, "<LinearParams>");
  int rows = 0, cols = 0;
  auto lin = kio::ReadFloatMatrix(is, binary, &rows, &cols);
  if (rows == 0 || cols == 0) throw std::runtime_error("AffineComponent: empty LinearParams");
  out_dim_ = rows;
  in_dim_ = cols;
  ExpectToken(is, binary, "<BiasParams>");
  auto b = kio::ReadFloatVector(is, binary);
  if ((int)b.size() != out_dim_) throw std::runtime_error("AffineComponent: bias size mismatch");
  std::string t = kio::ReadToken(is, binary);
  if (t == "<AvgInput>") {  // discarded
    kio::ReadFloatVector(is, binary);
    ExpectToken(is, binary, "<AvgInputCount>");
    kio::ReadFloat(is, binary);
    t = kio::ReadToken(is, binary);
  }
  is_gradient_ = false;
  if (t == "<IsGradient>") {
    is_gradient_ = kio::ReadBool(is, binary);
    t = kio::ReadToken(is, binary);
  }
  if (t != "</AffineComponent>") throw std::runtime_error("AffineComponent: bad token " + t);
  lin.insert(lin.end(), b.begin(), b.end());
  params_.ensure(sizeof(float) * lin.size());
  grad_.ensure(sizeof(float) * lin.size());
  h2d(params_.f(), lin.data(), (long)lin.size());
}
// ---------------------------------------------------------------------------
// Nnet
// ---------------------------------------------------------------------------
Nnet::~Nnet() {
  for (auto *c : components_) delete c;
}

void Nnet::Init(const std::string &config, Rng &rng) {
  std::istringstream is(config);
  std::string line;
  while (std::getline(is, line)) {
    auto hash = line.find('#');
    if (hash != std::string::npos) line = line.substr(0, hash);
    auto parts = split_ws(line);
    if (parts.empty()) continue;
    Component *c = Component::NewComponentOfType(parts[0]);
    if (!c) throw std::invalid_argument("Unknown component type " + parts[0] + " (not on the CTC path)");
    std::string args;
    for (size_t i = 1; i < parts.size(); i++) args += (i > 1 ? " " : "") + parts[i];
    c->InitFromString(args, rng);
    if (!components_.empty() && components_.back()->OutputDim() != c->InputDim()) {
      delete c;
      throw std::invalid_argument("dimension mismatch at component " + parts[0]);
    }
    components_.push_back(c);
  }
  if (components_.empty()) throw std::invalid_argument("empty nnet config");
}

int Nnet::LeftContext() const {  // nnet-nnet.cc:52-64
  int ans = 0;
  for (const Component *c : components_) ans += c->Context().front();
  return -ans;
}
int Nnet::RightContext() const {  // nnet-nnet.cc:66-73
  int ans = 0;
  for (const Component *c : components_) ans += c->Context().back();
  return ans;
}

int Nnet::FirstUpdatableComponent() const {  // nnet-nnet.cc:838-845
  for (int i = 0; i < NumComponents(); i++)
    if (components_[i]->IsUpdatable()) return i;
  return NumComponents();
}

int Nnet::LastUpdatableComponent() const {
  for (int i = NumComponents() - 1; i >= 0; i--)
    if (components_[i]->IsUpdatable()) return i;
  return -1;
}

void Nnet::SetComponent(int c, Component *component) {
  if (c < 0 || c >= NumComponents() || !component) {
    delete component;
    throw std::out_of_range("Nnet::SetComponent: bad index");
  }
  const bool in_ok = c == 0 || components_[c - 1]->OutputDim() == component->InputDim();
  const bool out_ok = c + 1 == NumComponents() || component->OutputDim() == components_[c + 1]->InputDim();
  if (!in_ok || !out_ok || (c > 0 && component->Context() != std::vector<int>{0})) {
    delete component;
    throw std::invalid_argument("Nnet::SetComponent: dimensions or context do not match the neighbours");
  }
  delete components_[c];
  components_[c] = component;
  // packed operands point into the replaced component's reserve
  for (Component *x : components_)
    if (auto *r = dynamic_cast<CuDNNRecurrentComponent *>(x)) r->ClearPackedInput();
}

void Nnet::ZeroStats() {
  for (auto *c : components_) c->ZeroStats();
}

void Nnet::SetMomentum(float m) {
  if (!(m >= 0.f && m < 1.f)) throw std::invalid_argument("momentum must be in [0, 1)");
  momentum_ = m;
  for (auto *c : components_) {
    if (c->IsUpdatable()) static_cast<UpdatableComponent *>(c)->SetMomentum(m);
    if (auto *cg = dynamic_cast<ClipGradientComponent *>(c)) cg->EnableShadow(m != 0.f);
  }
}

void Nnet::SetLearningRate(float lr) {
  for (auto *c : components_)
    if (c->IsUpdatable()) static_cast<UpdatableComponent *>(c)->SetLearningRate(lr);
}

// nnet-nnet.cc:170-183
void Nnet::Write(std::ostream &os, bool binary) const {
  WriteToken(os, binary, "<Nnet>");
  WriteToken(os, binary, "<NumComponents>");
  kio::WriteInt(os, binary, (int32_t)components_.size());
  WriteToken(os, binary, "<Components>");
  for (auto *c : components_) {
    c->Write(os, binary);
    if (!binary) os << "\n";
  }
  WriteToken(os, binary, "</Components>");
  WriteToken(os, binary, "</Nnet>");
}
// nnet-nnet.cc:185-220 (Component::ReadNew: "<Type>" token, then the body)
void Nnet::Read(std::istream &is, bool binary) {
  ExpectToken(is, binary, "<Nnet>");
  ExpectToken(is, binary, "<NumComponents>");
  const int n = kio::ReadInt(is, binary);
  if (n <= 0) throw std::runtime_error("Nnet::Read: <NumComponents> " + std::to_string(n));
  ExpectToken(is, binary, "<Components>");
  for (int i = 0; i < n; i++) components_.push_back(Component::ReadNew(is, binary));
  ExpectToken(is, binary, "</Components>");
  ExpectToken(is, binary, "</Nnet>");
  // Nnet::Read -> Check (nnet-nnet.cc:197-198, 281-289): every component's output feeds the next
  for (int i = 0; i < n; i++) {
    if (components_[i]->InputDim() <= 0 || components_[i]->OutputDim() <= 0)
      throw std::runtime_error("Nnet::Read: component " + std::to_string(i) + " has a non-positive dimension");
    if (i + 1 < n && components_[i]->OutputDim() != components_[i + 1]->InputDim())
      throw std::runtime_error("Nnet::Read: dimension mismatch between components " + std::to_string(i) + " (" +
                               components_[i]->Type() + ", output " + std::to_string(components_[i]->OutputDim()) +
                               ") and " + std::to_string(i + 1) + " (" + components_[i + 1]->Type() + ", input " +
                               std::to_string(components_[i + 1]->InputDim()) + ")");
  }
}
// ---------------------------------------------------------------------------
// NnetCtcUpdater (src/ctc/ctc-nnet-update.cc:76-348)
// ---------------------------------------------------------------------------
NnetCtcUpdater::NnetCtcUpdater(Nnet *nnet, bool update) : nnet_(nnet), update_(update) {}

static void set_minibatch(Nnet *nnet, int N) {  // Nnet::SetMiniBatch (nnet-nnet.cc:42-50)
  for (int c = 0; c < nnet->NumComponents(); c++) {
    auto *r = dynamic_cast<CuDNNRecurrentComponent *>(&nnet->GetComponent(c));
    if (r) r->SetMiniBatch(N);
  }
}

MinibatchStats NnetCtcUpdater::ComputeForMinibatch(const float *feats, int T_max, int N,
                                                   const int *num_frames, const int *flat_labels,
                                                   const int *label_lengths) {
  if (pending_) throw std::logic_error("ComputeForMinibatch with queued minibatches (Finish them first)");
  Enqueue(feats, T_max, N, num_frames, flat_labels, label_lengths);
  return Finish();
}

const CuMatrixBase &NnetCtcUpdater::Forward(const float *feats, int T_max, int N) {
  if (pending_) throw std::logic_error("Forward with queued minibatches (Finish them first)");
  if (N <= 0 || T_max <= 0) throw std::invalid_argument("empty minibatch");
  const int C = nnet_->NumComponents();
  set_minibatch(nnet_, N);
  err_word_.ensure(256);
  KCTC_HIP_CHECK(hipMemsetAsync(err_word_.p, 0, sizeof(unsigned), S()));
  for (int c = 0; c < C; c++)
    if (auto *r = dynamic_cast<CuDNNRecurrentComponent *>(&nnet_->GetComponent(c)))
      r->SetErrorWord(static_cast<unsigned *>(err_word_.p));
  forward_data_.resize(C + 1);
  SetupChunks(T_max, N);
  forward_data_[0].SetView(const_cast<float *>(feats), (long)T_max * N * nnet_->NumSplice(), nnet_->InputDim());
  Propagate(T_max, N);
  unsigned herr = 0;
  KCTC_HIP_CHECK(hipMemcpyAsync(&herr, err_word_.p, sizeof(unsigned), hipMemcpyDeviceToHost, S()));
  KCTC_HIP_CHECK(hipStreamSynchronize(S()));
  if (herr) throw std::runtime_error("recurrence hand-off timed out (device error word set)");
  return forward_data_[C];
}

void NnetCtcUpdater::Enqueue(const float *feats, int T_max, int N, const int *num_frames,
                             const int *flat_labels, const int *label_lengths) {
  if (pending_ == 2) throw std::logic_error("two minibatches already queued");
  const int C = nnet_->NumComponents();
  if (N <= 0 || T_max <= 0) throw std::invalid_argument("empty minibatch");
  const long rows = (long)T_max * N;
  set_minibatch(nnet_, N);
  // one error word per step for every recurrence: cleared here (stream order:
  // after the previous step's readback), read back at the end, and the
  // updates of a step that set it are skipped on the device
  err_word_.ensure(256);
  KCTC_HIP_CHECK(hipMemsetAsync(err_word_.p, 0, sizeof(unsigned), S()));
  if (inject_err_) {
    KCTC_HIP_CHECK(hipMemcpyAsync(err_word_.p, &inject_err_, sizeof(unsigned), hipMemcpyHostToDevice, S()));
    KCTC_HIP_CHECK(hipStreamSynchronize(S()));  // the source is a member that is reset next
    inject_err_ = 0;
  }
  for (int c = 0; c < C; c++)
    if (auto *r = dynamic_cast<CuDNNRecurrentComponent *>(&nnet_->GetComponent(c)))
      r->SetErrorWord(static_cast<unsigned *>(err_word_.p));
  forward_data_.resize(C + 1);
  SetupChunks(T_max, N);
  forward_data_[0].SetView(const_cast<float *>(feats), rows * nnet_->NumSplice(), nnet_->InputDim());
  Propagate(T_max, N);

  // ---- ComputeObjfAndDeriv (:171-259) with the warp-ctc ABI ----
  const CuMatrixBase &out = forward_data_[C];
  const int A = nnet_->OutputDim();
  for (int n = 0; n < N; n++)
    if (label_lengths[n] < 0) throw std::invalid_argument("negative label length");
  // input_lengths = NumFrames - ignore_frames (left_context + RightContext = 0 here)
  size_t ws = 0;
  {
    ctcOptions o;
    o.loc = CTC_GPU;
    o.stream = reinterpret_cast<ctcStream_t>(S());
    o.blank_label = 0;
    ctcStatus_t st = get_workspace_size(label_lengths, num_frames, A, N, o, &ws);
    if (st != CTC_STATUS_SUCCESS)
      throw std::runtime_error(std::string("get_workspace_size: ") + ctcGetStatusString(st));
    // size for the longest labels this T_max admits, once: a growing workspace
    // (label lengths vary per minibatch) would cost a device sync + realloc
    if (ws > ctc_ws_.bytes) {
      std::vector<int> worst_l(N, std::min(T_max, 639)), worst_t(N, T_max);
      size_t w2 = 0;
      if (get_workspace_size(worst_l.data(), worst_t.data(), A, N, o, &w2) == CTC_STATUS_SUCCESS)
        ws = std::max(ws, w2);
    }
  }
  ctc_ws_.ensure(ws);
  costs_dev_.ensure(sizeof(double) * N);
  ids_dev_.ensure(sizeof(int) * rows);
  CuMatrix &deriv = deriv_a_;
  deriv.Resize(rows, A);
  {
    ProfScope ps("layer_ctc");
    ctcStatus_t st = mictc_compute_ctc_loss_async(out.Data(), update_ ? deriv.Data() : nullptr,
                                                  flat_labels, label_lengths, num_frames, A, N,
                                                  static_cast<double *>(costs_dev_.p), ctc_ws_.p,
                                                  reinterpret_cast<ctcStream_t>(S()), 0);
    if (st != CTC_STATUS_SUCCESS)
      throw std::runtime_error(std::string("compute_ctc_loss: ") + ctcGetStatusString(st));
  }
  {
    ProfScope ps("argmax");
    row_argmax(S(), out.Data(), rows, A, static_cast<int *>(ids_dev_.p));  // FindRowMaxId
  }
  if (update_) Backprop(T_max, N);

  // ---- the single end-of-step device->host copy: costs, best-path ids,
  // the RNN components' device error words (into this slot's pinned buffer)
  Slot &sl = slots_[next_];
  const size_t need = sizeof(double) * N + sizeof(int) * rows + sizeof(unsigned) * C;
  if (need > sl.bytes) {
    if (sl.pinned) {
      if (sl.ev) KCTC_HIP_CHECK(hipEventSynchronize(sl.ev));
      (void)hipHostFree(sl.pinned);
    }
    KCTC_HIP_CHECK(hipHostMalloc((void **)&sl.pinned, need, hipHostMallocDefault));
    sl.bytes = need;
  }
  if (!sl.ev) KCTC_HIP_CHECK(hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming));
  double *hcost = reinterpret_cast<double *>(sl.pinned);
  int *hids = reinterpret_cast<int *>(sl.pinned + sizeof(double) * N);
  unsigned *herr = reinterpret_cast<unsigned *>(hids + rows);
  KCTC_HIP_CHECK(hipMemcpyAsync(hcost, costs_dev_.p, sizeof(double) * N, hipMemcpyDeviceToHost, S()));
  KCTC_HIP_CHECK(hipMemcpyAsync(hids, ids_dev_.p, sizeof(int) * rows, hipMemcpyDeviceToHost, S()));
  sl.nerr = 1;
  KCTC_HIP_CHECK(hipMemcpyAsync(herr, err_word_.p, sizeof(unsigned), hipMemcpyDeviceToHost, S()));
  KCTC_HIP_CHECK(hipEventRecord(sl.ev, S()));
  sl.N = N;
  sl.rows = rows;
  sl.num_frames.assign(num_frames, num_frames + N);
  long nlab = 0;
  for (int n = 0; n < N; n++) nlab += label_lengths[n];
  sl.labels.assign(flat_labels, flat_labels + nlab);
  sl.label_lengths.assign(label_lengths, label_lengths + N);
  next_ ^= 1;
  pending_++;
}

MinibatchStats NnetCtcUpdater::Finish() {
  if (!pending_) throw std::logic_error("no queued minibatch");
  Slot &sl = slots_[next_ ^ (pending_ == 2 ? 0 : 1)];  // the oldest
  pending_--;
  KCTC_HIP_CHECK(hipEventSynchronize(sl.ev));
  if (!pending_) CuDevice::Instantiate().Collect();  // no span of a later minibatch in flight
  const int N = sl.N;
  const long rows = sl.rows;
  const double *hcost = reinterpret_cast<const double *>(sl.pinned);
  const int *hids = reinterpret_cast<const int *>(sl.pinned + sizeof(double) * N);
  const unsigned *herr = reinterpret_cast<const unsigned *>(hids + rows);
  last_ids_.assign(hids, hids + rows);
  last_costs_.assign(hcost, hcost + N);
  for (int i = 0; i < sl.nerr; i++) {
    if (herr[i] & ~kErrPeerFailed) {
      // bits: 1 a recurrence's spin, 2 a streamed GEMM's wait, 8 a weight-gradient gate
      char what[64];
      snprintf(what, sizeof what, " (error word %d = 0x%x)", i, herr[i]);
      throw std::runtime_error(std::string("recurrence hand-off timed out") + what +
                               "; this minibatch's updates were skipped, the parameters are those before it");
    }
    if (herr[i])
      throw std::runtime_error("the step failed on another data-parallel rank; every rank skipped this "
                               "minibatch's updates, the parameters are those before it");
  }
  const int *num_frames = sl.num_frames.data(), *flat_labels = sl.labels.data();
  const int *label_lengths = sl.label_lengths.data();
  MinibatchStats st;
  for (int n = 0; n < N; n++) st.tot_objf += hcost[n];
  if (!(st.tot_objf == st.tot_objf)) throw std::runtime_error("costs sum is nan");  // :254
  // ---- ComputeTotAccuracy (:261-317) on the host ----
  const int blank = 0;
  long off = 0;
  double err = 0;
  std::vector<int> hyp;
  for (int n = 0; n < N; n++) {
    const int F = num_frames[n], L = label_lengths[n];
    hyp.assign((size_t)std::max(F, 0), 0);
    for (int i = 0; i < F; i++) hyp[i] = hids[(long)i * N + n];
    int i = 1, j = 1;
    while (j < F) {
      if (hyp[j] != hyp[j - 1] && hyp[j] != blank) hyp[i++] = hyp[j];
      j++;
    }
    hyp.resize(F > 0 ? i : 0);
    // LevenshteinEditDistance, unit costs
    err += levenshtein(flat_labels + off, L, hyp.data(), (int)hyp.size());
    st.tot_weight += L;
    off += L;
  }
  st.tot_accuracy = st.tot_weight - err;
  return st;
}

// Nnet::ComputeChunkInfo(num_splice, T*N) (nnet-nnet.cc:75-133) for the
// contiguous case: the last component's output is frame offset L (the
// network's left context), every component's input starts Context().front()
// frames earlier.  Rows: T*N*num_splice before a splicing component (the
// FormatNnetInput layout, ctc-nnet-update.cc:351-424), T*N after it; such a
// component must come first (the nnet2 CTC recipe's Splice).
void NnetCtcUpdater::SetupChunks(int T_max, int N) {
  const int C = nnet_->NumComponents();
  chunk_info_.resize(C + 1);
  int off = nnet_->LeftContext();
  for (int c = C; c >= 0; c--) {
    chunk_info_[c].num_chunks = N;
    chunk_info_[c].chunk_size = T_max;
    chunk_info_[c].feat_dim = c == 0 ? nnet_->InputDim() : nnet_->GetComponent(c - 1).OutputDim();
    chunk_info_[c].first_offset = off;
    if (c > 0) {
      const std::vector<int> ctx = nnet_->GetComponent(c - 1).Context();
      if (c - 1 > 0 && ctx != std::vector<int>{0})
        throw std::invalid_argument("a component with context other than {0} must come first (the recipe's Splice)");
      off += ctx.front();
    }
  }
}

void NnetCtcUpdater::Propagate(int T, int N) {  // :136-169
  const int C = nnet_->NumComponents();
  const CuDNNRecurrentComponent *below = nullptr;  // the last RNN, through identity components
  const int first = nnet_->FirstUpdatableComponent();
  for (int c = 0; c < C; c++) {
    const Component &comp = nnet_->GetComponent(c);
    if (const auto *r = dynamic_cast<const CuDNNRecurrentComponent *>(&comp)) {
      const void *rows = nullptr, *cols = nullptr;
      if (below && below->Desc().prec == r->Desc().prec) below->PackedOutput(&rows, &cols);
      r->SetPackedInput(rows, cols);
      // Backprop computes its input derivative (streamed dx GEMM): W^T packed now
      r->SetPrepackDx(update_ && c > first);
      r->SetPrepackW(update_ && c >= first);
      below = r;
    } else if (!comp.IsIdentityForward()) {
      below = nullptr;
    }
    const CuMatrixBase &in = forward_data_[c];
    CuMatrix &out = forward_data_[c + 1];
    if (comp.IsIdentityForward()) {
      out.SetView(in.Data(), in.NumRows(), comp.OutputDim());  // alias, no copy
      continue;
    }
    out.Resize((long)T * N, comp.OutputDim());
    // RNN -> identity-forward components -> RNN: the second one's input
    // projection streams off the first one's last recurrence
    const auto *rnn = dynamic_cast<const CuDNNRecurrentComponent *>(&comp);
    const CuDNNRecurrentComponent *next = nullptr;
    if (rnn) {
      int c2 = c + 1;
      while (c2 < C && nnet_->GetComponent(c2).IsIdentityForward()) c2++;
      if (c2 < C) next = dynamic_cast<const CuDNNRecurrentComponent *>(&nnet_->GetComponent(c2));
    }
    if (next) rnn->PropagateChained(in, &out, *next);
    else comp.Propagate(chunk_info_[c], chunk_info_[c + 1], in, &out);
  }
}

void NnetCtcUpdater::Backprop(int T, int N) {  // :320-348
  const int C = nnet_->NumComponents();
  const long rows = (long)T * N;
  const int A = nnet_->OutputDim();
  // deriv->Scale(-1) (:323)
  {
    ProfScope ps("scale");
    scale_inplace(S(), deriv_a_.Data(), rows * (long)A, -1.f);
  }
  CuMatrix *cur = &deriv_a_, *other = &deriv_b_;
  const int first = nnet_->FirstUpdatableComponent();
  int max_dim = A;
  for (int c = 0; c <= C; c++) max_dim = std::max(max_dim, chunk_info_[c].feat_dim);
  std::vector<int> updated;
  for (int c = C - 1; c >= first; c--) {
    Component &comp = nnet_->GetComponent(c);
    const CuMatrixBase &in = forward_data_[c], &outv = forward_data_[c + 1];
    Component *to_update = &comp;
    const bool need_in_deriv = c > first;
    CuMatrixBase *in_deriv = nullptr;
    CuMatrixBase view;
    if (need_in_deriv) {
      if (comp.IsIdentityForward()) {
        view = CuMatrixBase(cur->Data(), rows, comp.InputDim());  // in place
        in_deriv = &view;
      } else {
        other->Resize(rows, std::max(comp.InputDim(), max_dim));
        view = CuMatrixBase(other->Data(), rows, comp.InputDim());
        in_deriv = &view;
      }
    }
    if (auto *cg = dynamic_cast<ClipGradientComponent *>(&comp)) {
      cg->rng_ = &repair_rng_;  // RepairGradients draws RandUniform() from the process stream
      if (cg->Shadow()) to_update = cg->Shadow();  // momentum: delta_nnet's copy
    }
    const CuMatrixBase od(cur->Data(), rows, comp.OutputDim());
    const bool rec = exchange_ && dynamic_cast<CuDNNRecurrentComponent *>(&comp);
    if (rec) exchange_->BeforeRecurrence(S());
    comp.Backprop(chunk_info_[c], chunk_info_[c + 1], in, outv, od, to_update, in_deriv);
    if (rec) exchange_->AfterRecurrence();
    if (comp.IsUpdatable()) {
      auto *u = static_cast<UpdatableComponent *>(&comp);
      if (exchange_) exchange_->GradReady(c, u->GradData(), u->NumParameters(), u->GradStream());
      updated.push_back(c);
    }
    if (need_in_deriv && !comp.IsIdentityForward()) std::swap(cur, other);
  }
  CuDevice::Instantiate().Join();
  if (exchange_) exchange_->Finish();
  if (exchange_ && exchange_->WorldSize() > 1 && err_word_.p) {
    // the gradients just summed include every rank's: a step that failed on
    // ANY rank is skipped on all of them, so the replicas stay identical
    unsigned *err = static_cast<unsigned *>(err_word_.p);
    err_flag_.ensure(256);
    err_word_to_flag(S(), err, err_flag_.f());
    exchange_->AllReduceSum(err_flag_.f(), 1, S());
    flag_to_err_word(S(), err_flag_.f(), err);
  }
  for (int c : updated) {
    ProfScope ps("update");
    static_cast<UpdatableComponent *>(&nnet_->GetComponent(c))->ApplyUpdate(err_word_.p ? static_cast<const unsigned *>(err_word_.p) : nullptr);
  }
}

}  // namespace nnet2
}  // namespace kctc
