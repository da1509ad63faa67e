// nnet.h -- MI355X-native mirror of the reference's nnet2 CTC training path.
//
// Same class names and method meanings as the reference's nnet2 API
// (src/nnet2/nnet-component.h:157-348, nnet-cudnn-component.h, nnet-nnet.h,
// src/ctc/ctc-nnet-update.h), on device buffers and one HIP stream:
//   Component / UpdatableComponent      Propagate / Backprop / InitFromString /
//                                       Info / Read / Write / Copy / Vectorize /
//                                       SetZero / DotProduct / PerturbParams /
//                                       Scale / Add
//   SpliceComponent                     any sorted context, const-component-dim
//   CuDNNRecurrentComponent             -> rnn.hip (cuDNN-shaped gfx950 kernels)
//   ClipGradientComponent               -> elementwise.hip / clipgrad.hip
//   AffineComponent                     -> gemm.hip
//   Nnet                                component list, FirstUpdatableComponent
//   NnetCtcUpdater                      ComputeForMinibatch: forward, warp-ctc ABI
//                                       (ctc.hip), accuracy, backprop, SGD.
// Differences from the reference, all semantics-preserving:
//   * identity components (Splice context 0, ClipGradient forward) alias their
//     input instead of copying it;
//   * updates are applied after the whole backprop instead of inside each
//     component's Backprop; each component's input derivative is computed
//     before its update in the reference too, so the result is identical
//      and it leaves room for the RCCL gradient all-reduce;
//   * the first updatable component's input derivative (discarded by the
//     reference, FirstUpdatableComponent = 1) is not computed;
//   * the ~25 host synchronisations per minibatch of the reference (NaN-check
//     Sum()s, ApplyFloor counts, cost/id copies) become ONE end-of-step copy.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <iosfwd>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "clipgrad.h"
#include "glibc_rand.h"
#include "rnn.h"

namespace kctc {
namespace nnet2 {

// ---- minimal CuMatrix / ChunkInfo ------------------------------------------
struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  DevBuf(DevBuf &&o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; o.bytes = 0; }
  DevBuf &operator=(DevBuf &&o) noexcept {
    std::swap(p, o.p);
    std::swap(bytes, o.bytes);
    return *this;
  }
  ~DevBuf();
  void ensure(size_t b);  // grows (no copy), never shrinks
  float *f() const { return static_cast<float *>(p); }
};

class CuMatrixBase {
 public:
  CuMatrixBase() = default;
  CuMatrixBase(float *d, long r, int c) : data_(d), rows_(r), cols_(c) {}
  long NumRows() const { return rows_; }
  int NumCols() const { return cols_; }
  int Stride() const { return cols_; }
  float *Data() const { return data_; }

 protected:
  float *data_ = nullptr;
  long rows_ = 0;
  int cols_ = 0;
};

class CuMatrix : public CuMatrixBase {
 public:
  void Resize(long rows, int cols);  // kSetZero-free: contents undefined
  void SetView(float *d, long rows, int cols) { data_ = d; rows_ = rows; cols_ = cols; }

 private:
  DevBuf buf_;
};

struct ChunkInfo {  // src/nnet2/nnet-component.h:72-146 (contiguous case)
  int feat_dim = 0, num_chunks = 0, chunk_size = 0;
  int first_offset = 0;  // frame offset of a chunk's first row (Nnet::ComputeChunkInfo)
  long NumRows() const { return (long)num_chunks * chunk_size; }
  int NumCols() const { return feat_dim; }
  int NumChunks() const { return num_chunks; }
};

// Device/stream context (the role of CuDevice::Instantiate()).
struct CuDevice {
  int device = 0;
  hipStream_t stream = nullptr;
  // Lower-priority stream for the weight-gradient GEMMs, which then overlap
  // the next component's backward recurrence (nullptr: everything on `stream`).
  hipStream_t side = nullptr;
  // stream of the GEMMs that run concurrently with a recurrence and consume
  // its rows as they appear (streamed dx; nullptr: off)
  hipStream_t stream2 = nullptr;
  hipEvent_t fork_ev = nullptr, join_ev = nullptr;
  void Fork();  // side waits for the work queued so far on stream
  void Join();  // stream waits for the work queued so far on side
  // optional per-kernel-family timing (hipEvents on `stream` / `side`)
  bool profiling = false;
  struct Span { std::string family; hipEvent_t a, b; hipStream_t s; };
  std::vector<Span> spans;
  std::vector<size_t> open;  // indices of spans begun but not ended (LIFO)
  std::vector<hipEvent_t> pool;
  std::map<std::string, std::pair<double, int>> prof;  // family -> (ms, launches)
  void Begin(const char *family, hipStream_t s = nullptr);
  void End();
  void Collect();  // after a stream sync
  static CuDevice &Instantiate();
};

struct Rng {  // splitmix64 + Box-Muller (replaces Kaldi's rand()-based RandGauss)
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next();
  double uniform();  // (0, 1)
  double gauss();
};

// ---- components -------------------------------------------------------------
class Component {
 public:
  virtual ~Component() = default;
  virtual std::string Type() const = 0;
  virtual int InputDim() const = 0;
  virtual int OutputDim() const = 0;
  virtual void InitFromString(std::string args, Rng &rng) = 0;
  virtual std::string Info() const;
  virtual bool IsUpdatable() const { return false; }
  virtual bool IsIdentityForward() const { return false; }
  virtual bool BackpropNeedsInput() const { return true; }
  virtual bool BackpropNeedsOutput() const { return true; }
  virtual void Propagate(const ChunkInfo &in_info, const ChunkInfo &out_info,
                         const CuMatrixBase &in, CuMatrixBase *out) const = 0;
  // in_deriv may alias out_deriv (in-place) or be nullptr (not needed).
  virtual void Backprop(const ChunkInfo &in_info, const ChunkInfo &out_info,
                        const CuMatrixBase &in_value, const CuMatrixBase &out_value,
                        const CuMatrixBase &out_deriv, Component *to_update,
                        CuMatrixBase *in_deriv) const = 0;
  virtual void Write(std::ostream &os, bool binary) const = 0;
  virtual void Read(std::istream &is, bool binary) = 0;
  // a deep copy (device parameters and statistics copied on the stream); like
  // the reference's copy constructors it carries no minibatch state, so a
  // copied CuDNNRecurrentComponent must Propagate before it can Backprop
  virtual Component *Copy() const = 0;
  virtual void ZeroStats() {}
  // frame offsets this component reads relative to each output frame
  // (nnet-component.h:188; only SpliceComponent has more than {0})
  virtual std::vector<int> Context() const { return std::vector<int>(1, 0); }
  static Component *NewComponentOfType(const std::string &type);
  // "<Type>" token, then the body (nnet-component.cc:38-48)
  static Component *ReadNew(std::istream &is, bool binary);
};

class UpdatableComponent : public Component {
 public:
  bool IsUpdatable() const override { return true; }
  float LearningRate() const { return learning_rate_; }
  void SetLearningRate(float lr) { learning_rate_ = lr; }
  // nnet-component.h:295-318.  Both updatable components on this path keep
  // all their parameters in ParamData() (Vectorize order), so these are
  // defined once on that flat vector; each equals the reference's per-class
  // definition (AffineComponent: TraceMatMat(linear, other.linear, kTrans) +
  // VecVec(bias, other.bias) == the flat dot, nnet-component.cc:1026-1123;
  // CuDNNRecurrentComponent: filter_params_, nnet-cudnn-component.cc:723-772).
  // SetZero(true): parameters 0, learning rate 1, is-gradient (then a Backprop
  // with this as to_update followed by ApplyUpdate stores the gradient in it)
  virtual void SetZero(bool treat_as_gradient);
  // fp64 accumulation on the device (the reference: fp32 VecVec)
  virtual double DotProduct(const UpdatableComponent &other) const;
  // params += stddev * N(0,1), from the process's perturbation stream
  // (SetPerturbSeed; each call draws fresh noise)
  virtual void PerturbParams(float stddev);
  virtual void Scale(float scale);
  virtual void Add(float alpha, const UpdatableComponent &other);
  bool IsGradient() const { return is_gradient_; }
  static void SetPerturbSeed(unsigned long long seed);
  virtual long NumParameters() const = 0;
  virtual void Vectorize(float *host) const = 0;      // host copy of all params
  virtual void UnVectorize(const float *host) = 0;
  // gradient produced by the last Backprop (device), in Vectorize order
  virtual float *GradData() = 0;
  // the parameters (device), in Vectorize order
  virtual float *ParamData() = 0;
  // stream on which GradData() was produced (the exchange waits on it)
  hipStream_t GradStream() const;
  // forget the stream of the last Backprop (standalone components: the
  // Backprop's stream belongs to the calling handle, which may go first)
  void ResetGradStream() { grad_stream_ = nullptr; }
  // params += lr * (clipped) grad; skipped on device when *skip != 0 (the
  // step's recurrence hand-off failed: its gradients are not trusted)
  virtual void ApplyUpdate(const unsigned *skip = nullptr) = 0;
  // TrainNnetSimple momentum (ctc-nnet-train.cc:194-245): the update goes to
  // a delta copy (delta += lr * clip(grad)), then params += delta and
  // delta *= momentum.  0 = plain SGD (the recipe's default).
  void SetMomentum(float m);
  float Momentum() const { return momentum_; }

 protected:
  void UpdateWith(float *params, const float *grad, float clip, const unsigned *skip);
  void CopyUpdatableFrom(const UpdatableComponent &o);  // learning rate, is-gradient
  void CheckSameKind(const UpdatableComponent &o, const char *what) const;
  float learning_rate_ = 0.001f;
  bool is_gradient_ = false;  // <IsGradient>, read and written back
  hipStream_t grad_stream_ = nullptr;  // nullptr: the device's compute stream
  float momentum_ = 0.f;
  DevBuf delta_;
};

// SpliceComponent (nnet-component.cc:2504-2820).  Its input is the
// FormatNnetInput layout for num_splice = 1 + LeftContext + RightContext:
// output frame j (= t*N + n) owns input rows j*num_splice .. +num_splice-1
// (frames t .. t+num_splice-1 of utterance n), and output block c copies row
// j*num_splice + L + context[c] (L = the network's left context; the
// reference's CopyRows with ChunkInfo(num_splice, T*N), :2606-2689); the last
// const-component-dim columns come from the chunk's first row.  Context {0}
// without a const part (the CTC recipe's) aliases its input.
class SpliceComponent : public Component {
 public:
  std::string Type() const override { return "SpliceComponent"; }
  int InputDim() const override { return input_dim_; }
  int OutputDim() const override { return (input_dim_ - const_dim_) * (int)context_.size() + const_dim_; }
  void InitFromString(std::string args, Rng &rng) override;
  bool IsIdentityForward() const override { return context_ == std::vector<int>{0} && const_dim_ == 0; }
  std::vector<int> Context() const override { return context_; }
  bool BackpropNeedsInput() const override { return false; }
  bool BackpropNeedsOutput() const override { return false; }
  void Propagate(const ChunkInfo &, const ChunkInfo &, const CuMatrixBase &in,
                 CuMatrixBase *out) const override;
  void Backprop(const ChunkInfo &, const ChunkInfo &, const CuMatrixBase &, const CuMatrixBase &,
                const CuMatrixBase &, Component *, CuMatrixBase *) const override;
  void Write(std::ostream &os, bool binary) const override;
  void Read(std::istream &is, bool binary) override;
  Component *Copy() const override;

 private:
  void Init(int input_dim, std::vector<int> context, int const_dim);
  int input_dim_ = 0, const_dim_ = 0;
  std::vector<int> context_{0};
};

class CuDNNRecurrentComponent : public UpdatableComponent {
 public:
  CuDNNRecurrentComponent();
  ~CuDNNRecurrentComponent() override;
  std::string Type() const override { return "CuDNNRecurrentComponent"; }
  int InputDim() const override { return desc_.D; }
  int OutputDim() const override { return desc_.H * desc_.dirs; }
  void InitFromString(std::string args, Rng &rng) override;
  std::string Info() const override;
  void Propagate(const ChunkInfo &in_info, const ChunkInfo &out_info, const CuMatrixBase &in,
                 CuMatrixBase *out) const override;
  void Backprop(const ChunkInfo &in_info, const ChunkInfo &out_info,
                const CuMatrixBase &in_value, const CuMatrixBase &out_value,
                const CuMatrixBase &out_deriv, Component *to_update,
                CuMatrixBase *in_deriv) const override;
  void Write(std::ostream &os, bool binary) const override;
  void Read(std::istream &is, bool binary) override;
  Component *Copy() const override;
  void SetZero(bool treat_as_gradient) override;
  long NumParameters() const override { return desc_.params_size(); }
  void Vectorize(float *host) const override;
  void UnVectorize(const float *host) override;
  float *GradData() override { return grad_.f(); }
  float *ParamData() override {  // (a writer: the forward's packed W^T goes stale)
    ++pver_;
    return params_.f();
  }
  void ApplyUpdate(const unsigned *skip = nullptr) override;
  // the updater marks the RNNs whose Backprop computes an input derivative:
  // their forward packs W^T for it on the side stream (rnn.h RnnPrepack)
  void SetPrepackDx(bool on) const { prepack_dx_ = on; }
  // ... and the RNNs it updates: their forward packs x^T / y^T for the weight
  // GEMMs on the side stream (RnnPrepack::wgrad)
  void SetPrepackW(bool on) const { prepack_w_ = on; }
  // device error word of the recurrences (hand-off timeout); the updater
  // points every RNN at its own per-step word (SetErrorWord)
  unsigned *DeviceError() const { return err_ext_ ? err_ext_ : err_; }
  void SetErrorWord(unsigned *e) const { err_ext_ = e; }
  // workgroup cap of the side-stream weight GEMMs: the CUs left over by the
  // backward recurrence
  int side_gemm_blocks() const;
  const RnnPrepack *wgrad_prepack(const CuMatrixBase &in_value, const CuMatrixBase &out_value) const;
  const RnnDesc &Desc() const { return desc_; }
  // arithmetic of the recurrences and gate GEMMs (rnn.h RnnDesc::prec); the
  // parameters and the model file stay fp32
  void SetPrecision(int prec) {
    if (prec == 1 && desc_.mode != kLstm && desc_.mode != kGru)
      throw std::invalid_argument("bf16 products exist for LSTM / GRU only");
    rnn_set_precision(desc_, prec);
  }
  void SetMiniBatch(int n) const { mini_batch_ = n; }  // Init(mini_batch) on change
  // whether the last Propagate ran on a T x N input (Backprop's reserve-space precondition)
  bool PropagatedShape(int T, int N) const { return seq_length_ == T && mini_batch_ == N && reserve_.p; }
  // Propagate whose last recurrence also produces `next`'s layer-0 input
  // projection on the side stream (rnn.h RnnFwdChain), `next` being the
  // following RNN with only identity-forward components in between; `next`
  // then skips that projection in its own Propagate.
  void PropagateChained(const CuMatrixBase &in, CuMatrixBase *out, const CuDNNRecurrentComponent &next) const;
  // bf16 one-layer bidirectional components write their output also as the
  // packed bf16 GEMM operands (rnn.h rnn_packed_output); the next RNN reads
  // them instead of packing its input (set by the updater from the RNN below,
  // through identity components; nullptrs: pack)
  bool PackedOutput(const void **rows, const void **cols) const;
  void SetPackedInput(const void *rows, const void *cols) const {
    in_rows_ = rows;
    in_cols_ = cols;
    in_tn_[0] = in_tn_[1] = -1;  // bound to a shape by the next Propagate
  }
  // the component below changed (Nnet::SetComponent): its packed output is gone
  void ClearPackedInput() const { SetPackedInput(nullptr, nullptr); }

 private:
  void Init(Rng &rng);
  RnnDesc desc_;
  int max_seq_length_ = 2000;
  float param_stddev_ = 0.02f, bias_stddev_ = 0.2f, clip_gradient_ = 5.0f;
  DevBuf params_, grad_;
  mutable DevBuf reserve_, workspace_;
  mutable int mini_batch_ = 0, seq_length_ = 0;
  mutable bool input_projected_ = false;  // set by the previous component's PropagateChained
  mutable float input_bound_ = 0.f;       // ditto: bound on |input| (0: unknown)
  mutable const void *in_rows_ = nullptr, *in_cols_ = nullptr;  // SetPackedInput
  mutable int in_tn_[2] = {-1, -1};  // (T, N) of the Propagate that read in_rows_ / in_cols_
  const void *packed_input_cols(int T, int N) const {  // Backprop: only for the pass they were set for
    return in_tn_[0] == T && in_tn_[1] == N ? in_cols_ : nullptr;
  }
  unsigned *err_ = nullptr;
  mutable unsigned *err_ext_ = nullptr;
  // W^T packed by the last forward (RnnPrepack) for parameter version pre_ver_
  mutable bool prepack_dx_ = false, prepack_w_ = false;
  mutable RnnPrepack pre_;
  mutable const float *pre_x_ = nullptr, *pre_y_ = nullptr;  // the forward's input / output (pre_.wdone)
  mutable unsigned pre_ver_ = 0;
  unsigned pver_ = 1;  // bumped by every parameter write
  void Forward(const CuMatrixBase &in, CuMatrixBase *out, RnnFwdChain *chain) const;
};

class ClipGradientComponent : public Component {
 public:
  ClipGradientComponent();
  ~ClipGradientComponent() override;
  std::string Type() const override { return "ClipGradientComponent"; }
  int InputDim() const override { return dim_; }
  int OutputDim() const override { return dim_; }
  void InitFromString(std::string args, Rng &rng) override;
  std::string Info() const override;
  bool IsIdentityForward() const override { return true; }
  bool BackpropNeedsOutput() const override { return false; }
  void Propagate(const ChunkInfo &, const ChunkInfo &, const CuMatrixBase &in,
                 CuMatrixBase *out) const override;
  void Backprop(const ChunkInfo &, const ChunkInfo &, const CuMatrixBase &in_value,
                const CuMatrixBase &, const CuMatrixBase &out_deriv, Component *to_update,
                CuMatrixBase *in_deriv) const override;
  void Write(std::ostream &os, bool binary) const override;
  void Read(std::istream &is, bool binary) override;
  Component *Copy() const override;
  void ZeroStats() override;
  // the counters' Scale / Add (nnet-cudnn-component.cc:1064-1073)
  void Scale(float scale);
  void Add(float alpha, const ClipGradientComponent &other);
  // host view of the device counters (valid after a stream sync)
  void SyncStats() const;
  double NumClipped() const { return num_clipped_; }
  double Count() const { return count_; }
  // the process's rand() stream (NnetCtcUpdater's, seeded by --srand): the
  // RandUniform() of RepairGradients is drawn from it during Backprop, only
  // when the reference's short-circuit conditions get that far (:988-991)
  mutable GlibcRand *rng_ = nullptr;
  // momentum training passes delta_nnet's copy as to_update: counters go to
  // the copy, the repair decision reads this component's own counters
  void EnableShadow(bool on);
  ClipGradientComponent *Shadow() const { return shadow_; }


 private:
  int dim_ = 0;
  float clipping_threshold_ = 15.0f;
  bool norm_based_clipping_ = false;
  float self_repair_clipped_proportion_threshold_ = 0.01f, self_repair_target_ = 0.0f,
        self_repair_scale_ = 1.0f;
  mutable double num_clipped_ = 0, count_ = 0, num_self_repaired_ = 0, num_backpropped_ = 0;
  ClipState *dev_ = nullptr;
  mutable DevBuf scratch_;
  ClipGradientComponent *shadow_ = nullptr;
};

// SoftmaxComponent (nnet-component.cc:929-946): the output layer the recipe
// appends for decoding (egs/wsj/s5/steps/ctc/train.sh:471-477); forward only
// on this path (CTC training runs on the un-normalised affine output).
// The NonlinearComponent statistics are kept for the model file.
class SoftmaxComponent : public Component {
 public:
  std::string Type() const override { return "SoftmaxComponent"; }
  int InputDim() const override { return dim_; }
  int OutputDim() const override { return dim_; }
  void InitFromString(std::string args, Rng &rng) override;
  bool BackpropNeedsInput() const override { return false; }
  void Propagate(const ChunkInfo &, const ChunkInfo &, const CuMatrixBase &in,
                 CuMatrixBase *out) const override;
  // DiffSoftmaxPerRow; to_update's statistics get UpdateStats(out_value)
  // (nnet-component.cc:948-976, NonlinearComponent::UpdateStats)
  void Backprop(const ChunkInfo &, const ChunkInfo &, const CuMatrixBase &, const CuMatrixBase &out_value,
                const CuMatrixBase &out_deriv, Component *to_update, CuMatrixBase *in_deriv) const override;
  void Write(std::ostream &os, bool binary) const override;
  void Read(std::istream &is, bool binary) override;
  Component *Copy() const override;
  // NonlinearComponent::Scale / Add of the statistics (nnet-am-average)
  void Scale(float scale);
  void Add(float alpha, const SoftmaxComponent &other);
  const std::vector<double> &ValueSum() const { return value_sum_; }
  double Count() const { return count_; }

 private:
  int dim_ = 0;
  mutable DevBuf ws_;
  std::vector<double> value_sum_, deriv_sum_;
  double count_ = 0;
};

class AffineComponent : public UpdatableComponent {
 public:
  std::string Type() const override { return "AffineComponent"; }
  int InputDim() const override { return in_dim_; }
  int OutputDim() const override { return out_dim_; }
  void InitFromString(std::string args, Rng &rng) override;
  std::string Info() const override;
  bool BackpropNeedsOutput() const override { return false; }
  void Propagate(const ChunkInfo &, const ChunkInfo &, const CuMatrixBase &in,
                 CuMatrixBase *out) const override;
  void Backprop(const ChunkInfo &, const ChunkInfo &, const CuMatrixBase &in_value,
                const CuMatrixBase &, const CuMatrixBase &out_deriv, Component *to_update,
                CuMatrixBase *in_deriv) const override;
  void Write(std::ostream &os, bool binary) const override;
  void Read(std::istream &is, bool binary) override;
  Component *Copy() const override;
  long NumParameters() const override { return (long)(in_dim_ + 1) * out_dim_; }
  void Vectorize(float *host) const override;  // linear (row-major) then bias
  void UnVectorize(const float *host) override;
  float *GradData() override { return grad_.f(); }
  float *ParamData() override { return params_.f(); }
  void ApplyUpdate(const unsigned *skip = nullptr) override;

 private:
  int in_dim_ = 0, out_dim_ = 0;
  DevBuf params_, grad_;  // [out][in] followed by [out]
  mutable DevBuf ws_;
};

// ---- Nnet / updater ---------------------------------------------------------
class Nnet {
 public:
  ~Nnet();
  void Init(const std::string &config, Rng &rng);
  int NumComponents() const { return (int)components_.size(); }
  Component &GetComponent(int c) { return *components_[c]; }
  const Component &GetComponent(int c) const { return *components_[c]; }
  int FirstUpdatableComponent() const;
  int LastUpdatableComponent() const;  // -1 when none (nnet-nnet.cc)
  // takes ownership; dimensions must still chain (nnet-nnet.cc:659-665)
  void SetComponent(int c, Component *component);
  // Nnet::LeftContext / RightContext (nnet-nnet.cc:52-73): the sums of the
  // components' first (negated) and last context offsets
  int LeftContext() const;
  int RightContext() const;
  int NumSplice() const { return 1 + LeftContext() + RightContext(); }
  int InputDim() const { return components_.front()->InputDim(); }
  int OutputDim() const { return components_.back()->OutputDim(); }
  void ZeroStats();
  void SetLearningRate(float lr);
  void SetMomentum(float m);
  float Momentum() const { return momentum_; }
  void Write(std::ostream &os, bool binary) const;
  void Read(std::istream &is, bool binary);

 private:
  std::vector<Component *> components_;
  float momentum_ = 0.f;
};

// Data-parallel gradient exchange (RCCL over xGMI); implemented in dp.cpp.
class GradExchange {
 public:
  virtual ~GradExchange() = default;
  virtual void GradReady(int component, float *grad, long n, hipStream_t producer) = 0;
  // around the Backprop of a component that launches a backward recurrence:
  // Before (the compute stream may be made to wait for exchange work already
  // queued), After (the recurrence is enqueued: exchange work may be queued
  // behind its residency, rnn.h rnn_comm_gate)
  virtual void BeforeRecurrence(hipStream_t compute) { (void)compute; }
  virtual void AfterRecurrence() {}
  virtual void Finish() = 0;  // compute stream waits for every launched all-reduce
  virtual int WorldSize() const = 0;
  // in-place sum of buf over the ranks, ordered on stream s (s waits for it)
  virtual void AllReduceSum(float *buf, long n, hipStream_t s) = 0;
};

struct MinibatchStats {
  double tot_objf = 0, tot_accuracy = 0, tot_weight = 0;
};

// kaldi::LevenshteinEditDistance (unit costs), bit-parallel (nnet.cpp)
int levenshtein(const int *ref, int m, const int *hyp, int n);

class NnetCtcUpdater {
 public:
  NnetCtcUpdater(Nnet *nnet, bool update);
  // feats: device [T_max*N][input_dim] (FormatNnetInput layout)
  MinibatchStats ComputeForMinibatch(const float *feats, int T_max, int N, const int *num_frames,
                                     const int *flat_labels, const int *label_lengths);
  // The same split in two: Enqueue queues all device work of a minibatch and
  // the asynchronous readback of its costs, best paths and device error
  // words (at most two minibatches in flight); Finish waits for the oldest
  // one and computes its stats (ComputeTotAccuracy on the host).  With one
  // minibatch queued ahead the host's per-step work (readback, accuracy,
  // the caller's loop, the next step's launches) overlaps the device's.
  void Enqueue(const float *feats, int T_max, int N, const int *num_frames, const int *flat_labels,
               const int *label_lengths);
  int Pending() const { return pending_; }
  MinibatchStats Finish();
  void SetExchange(GradExchange *ex) { exchange_ = ex; }
  // NnetComputation (src/nnet2/nnet-compute.cc): forward only, N sequences
  // time-major; the output stays valid until the next minibatch
  const CuMatrixBase &Forward(const float *feats, int T_max, int N);
  // best-path ids ([T_max*N], FindRowMaxId) of the last minibatch Finish()ed
  const std::vector<int> &LastBestPath() const { return last_ids_; }
  // per-utterance CTC costs (-log p, warp-ctc `costs`) of that minibatch
  const std::vector<double> &LastCosts() const { return last_costs_; }
  // network output of the last minibatch queued (device, [T_max*N][A])
  const CuMatrixBase &Output() const { return forward_data_.empty() ? empty_ : forward_data_.back(); }
  // srand(seed) of the process stream (nnet2-ctc-train-simple.cc:47,69;
  // default 0) that ClipGradient self-repair draws from
  void Srand(unsigned seed) { repair_rng_.Seed(seed); }
  long RandCalls() const { return repair_rng_.Calls(); }
  // test hook: the next minibatch's device error word starts as `word` (as if
  // a recurrence had timed out), so its updates are skipped and Finish throws
  void InjectStepError(unsigned word) { inject_err_ = word; }

 private:
  void SetupChunks(int T_max, int N);
  void Propagate(int T, int N);
  void Backprop(int T, int N);
  Nnet *nnet_;
  bool update_;
  GradExchange *exchange_ = nullptr;
  GlibcRand repair_rng_{0};
  std::vector<CuMatrix> forward_data_;
  std::vector<int> last_ids_;
  std::vector<double> last_costs_;
  CuMatrixBase empty_;
  std::vector<ChunkInfo> chunk_info_;
  CuMatrix deriv_a_, deriv_b_;
  DevBuf ctc_ws_, costs_dev_, ids_dev_;
  DevBuf err_word_;  // this step's recurrence error word (all RNNs), cleared per step
  DevBuf err_flag_;  // the word as a 0/1 float, summed over the data-parallel ranks
  unsigned inject_err_ = 0;
  struct Slot {  // one minibatch in flight: pinned readback + what its stats need
    char *pinned = nullptr;
    size_t bytes = 0;
    hipEvent_t ev = nullptr;
    int N = 0, nerr = 0;
    long rows = 0;
    std::vector<int> num_frames, labels, label_lengths;
  };
  Slot slots_[2];
  int next_ = 0, pending_ = 0;
};

}  // namespace nnet2
}  // namespace kctc
