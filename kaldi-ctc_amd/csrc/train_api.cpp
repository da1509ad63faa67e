// train_api.cpp -- C ABI of include/kaldi_ctc_train.h: the nnet2 trainer,
// RCCL data parallelism, FormatNnetInput and the synthetic minibatch generator.
#include "kaldi_ctc_train.h"
#include "kaldi_ctc_decode.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "common.h"
#include "decodable.h"
#include "egs.h"
#include "elementwise.h"
#include "kaldi_io.h"
#include "nnet.h"
#include "nnet_handle.h"

using kctc::nnet2::CuDevice;

int kctc_usable_cus_override();

namespace {

thread_local std::string g_err;

// Gradient all-reduce over RCCL on a dedicated stream: each component's
// gradient bucket is reduced as soon as its Backprop has produced it, while
// the compute stream goes on with the layers below (overlap); the SGD updates
// wait for the last bucket.  Sum semantics: the summed gradient of the G
// per-rank minibatches equals the gradient of their concatenation, then the
// reference's per-component clip (+-clip-gradient) and SGD run identically
// on every rank, so replicas stay bit-identical.
//
// CU budget: the all-reduces run during the backward pass,
// beside the persistent recurrence and the streamed dx GEMM, whose blocks must
// all be resident.  RCCL's kernels are capped at kctc_comm_ctas() blocks
// (ncclConfig_t.maxCTAs) and the streamed GEMMs leave that many CUs free
// (rnn_set_cu_budget), so even if every RCCL block kept a CU to itself the
// recurrence's workgroups still find theirs.
int kctc_comm_ctas() {
  const char *e = getenv("KCTC_COMM_CTAS");
  const int v = e && *e ? atoi(e) : 16;
  return std::max(1, std::min(v, 64));
}

// Residency-gated exchange: a bucket's reduction is queued on
// the comm stream only behind the NEXT backward recurrence's launch, after a
// gate kernel's wait until every workgroup of that recurrence is resident
// (rnn_comm_gate, its blocks off the recurrence's XCDs; after its end instead
// when it uses scratch, rnn.h rnn_last_bwd_scratch_free), and the launch of the recurrence after that waits
// for it.  So no exchange kernel holds a CU while a recurrence's workgroups
// are being placed -- the condition under which an XCD-pinned recurrence
// (which needs all CUs of its XCDs) could wait on an all-reduce that waits on
// another GPU -- and the backward recurrences stay XCD-pinned with the
// exchange configured (rnn_set_comm_gated).  The last bucket (bottom
// component) goes out at Finish, with no recurrence after it.  KCTC_COMM_GATE=0
// reduces every bucket at once and leaves the backward unpinned (round 3).
class GatedExchange : public kctc::nnet2::GradExchange {
 public:
  GatedExchange(hipStream_t compute, int comm_cus) : compute_(compute) {
    const char *e = getenv("KCTC_COMM_GATE");
    gated_ = !(e && *e == '0');
    // the gate waits on the device's registration word, which every network's
    // backward recurrences add to: two gated exchanges on one device would
    // wait on each other's recurrences
    if (gated_ && kctc::rnn_comm_gated())
      throw std::runtime_error("a gated gradient exchange is already active on this device (one data-parallel "
                               "network per device and process; KCTC_COMM_GATE=0 lifts the limit)");
    kctc::rnn_set_cu_budget(kctc_usable_cus_override(), comm_cus);
    if (gated_) kctc::rnn_set_comm_gated(true);
    KCTC_HIP_CHECK(hipStreamCreateWithFlags(&comm_stream_, hipStreamNonBlocking));
    KCTC_HIP_CHECK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
    KCTC_HIP_CHECK(hipEventCreateWithFlags(&after_, hipEventDisableTiming));
  }
  ~GatedExchange() override {
    kctc::rnn_set_cu_budget(kctc_usable_cus_override(), 0);
    if (gated_) kctc::rnn_set_comm_gated(false);
    (void)hipStreamSynchronize(comm_stream_);
    (void)hipStreamDestroy(comm_stream_);
    (void)hipEventDestroy(done_);
    (void)hipEventDestroy(after_);
    for (auto ev : pool_) (void)hipEventDestroy(ev);
  }
  void GradReady(int, float *grad, long n, hipStream_t producer) override {
    if (next_ev_ == pool_.size()) {
      hipEvent_t ev;
      KCTC_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      pool_.push_back(ev);
    }
    hipEvent_t ev = pool_[next_ev_++];
    KCTC_HIP_CHECK(hipEventRecord(ev, producer));
    pending_.push_back({grad, n, ev});
    if (!gated_) Launch();
  }
  void BeforeRecurrence(hipStream_t compute) override {
    // the reductions queued behind the previous recurrence ran while it was
    // resident; this launch waits for them (they normally end long before)
    if (gated_ && launched_) KCTC_HIP_CHECK(hipStreamWaitEvent(compute, done_, 0));
    launched_ = false;
  }
  void AfterRecurrence() override {
    if (!gated_ || pending_.empty()) return;
    if (kctc::rnn_last_bwd_scratch_free()) {
      kctc::rnn_comm_gate(comm_stream_, kctc::rnn_bwd_registrations());
    } else {  // nothing beside a recurrence that uses scratch: after its end
      KCTC_HIP_CHECK(hipEventRecord(after_, compute_));
      KCTC_HIP_CHECK(hipStreamWaitEvent(comm_stream_, after_, 0));
    }
    Launch();
  }
  void Finish() override {
    Launch();
    KCTC_HIP_CHECK(hipEventRecord(done_, comm_stream_));
    KCTC_HIP_CHECK(hipStreamWaitEvent(compute_, done_, 0));
    launched_ = false;
    next_ev_ = 0;
  }
  void AllReduceSum(float *buf, long n, hipStream_t s) override {
    KCTC_HIP_CHECK(hipEventRecord(done_, s));
    KCTC_HIP_CHECK(hipStreamWaitEvent(comm_stream_, done_, 0));
    Reduce(buf, n);
    KCTC_HIP_CHECK(hipEventRecord(done_, comm_stream_));
    KCTC_HIP_CHECK(hipStreamWaitEvent(s, done_, 0));
  }

 protected:
  virtual void Reduce(float *buf, long n) = 0;  // in place on comm_stream_
  hipStream_t compute_, comm_stream_ = nullptr;

 private:
  void Launch() {
    if (pending_.empty()) return;
    for (const auto &b : pending_) {
      KCTC_HIP_CHECK(hipStreamWaitEvent(comm_stream_, b.ready, 0));
      Reduce(b.grad, b.n);
    }
    pending_.clear();
    KCTC_HIP_CHECK(hipEventRecord(done_, comm_stream_));
    launched_ = true;
  }
  struct Bucket {
    float *grad;
    long n;
    hipEvent_t ready;
  };
  bool gated_ = true, launched_ = false;
  hipEvent_t done_ = nullptr;
  hipEvent_t after_ = nullptr;  // the end of a recurrence that uses scratch
  std::vector<hipEvent_t> pool_;
  size_t next_ev_ = 0;
  std::vector<Bucket> pending_;
};

class RcclExchange : public GatedExchange {
 public:
  RcclExchange(const void *uid, int rank, int world, hipStream_t compute)
      : GatedExchange(compute, kctc_comm_ctas()), world_(world) {
    ncclUniqueId id;
    memcpy(&id, uid, sizeof(id));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 1;
    cfg.maxCTAs = kctc_comm_ctas();
    cfg.minCTAs = std::min(cfg.maxCTAs, 4);
    if (ncclCommInitRankConfig(&comm_, world, id, rank, &cfg) != ncclSuccess)
      throw std::runtime_error("ncclCommInitRankConfig failed");
  }
  ~RcclExchange() override {
    (void)hipStreamSynchronize(comm_stream_);
    ncclCommDestroy(comm_);
  }
  int WorldSize() const override { return world_; }

 protected:
  void Reduce(float *buf, long n) override {
    if (ncclAllReduce(buf, buf, (size_t)n, ncclFloat, ncclSum, comm_, comm_stream_) != ncclSuccess)
      throw std::runtime_error("ncclAllReduce failed");
  }

 private:
  int world_;
  ncclComm_t comm_ = nullptr;
};

// The same exchange over a host transport (kctc_nnet_enable_dp_host): the
// buckets are registered in backprop order as with RCCL; Finish() sums each
// one through the caller's all-reduce (device -> pinned host -> all-reduce ->
// device) before the updates.  Host-synchronous: a transport for ranks that
// share a GPU or have no RCCL peer, not the fast path.
class HostExchange : public kctc::nnet2::GradExchange {
 public:
  HostExchange(kctc_host_allreduce_fn fn, void *user, int world, hipStream_t compute)
      : fn_(fn), user_(user), world_(world), compute_(compute) {
    KCTC_HIP_CHECK(hipEventCreateWithFlags(&ev_, hipEventDisableTiming));
  }
  ~HostExchange() override {
    if (host_) (void)hipHostFree(host_);
    (void)hipEventDestroy(ev_);
  }
  void GradReady(int, float *grad, long n, hipStream_t producer) override {
    buckets_.push_back({grad, n, producer});
  }
  void Finish() override {
    for (const auto &b : buckets_) {
      if ((size_t)b.n > cap_) {
        if (host_) KCTC_HIP_CHECK(hipHostFree(host_));
        KCTC_HIP_CHECK(hipHostMalloc((void **)&host_, sizeof(float) * b.n, hipHostMallocDefault));
        cap_ = (size_t)b.n;
      }
      KCTC_HIP_CHECK(hipEventRecord(ev_, b.producer));
      KCTC_HIP_CHECK(hipStreamWaitEvent(compute_, ev_, 0));
      KCTC_HIP_CHECK(hipMemcpyAsync(host_, b.grad, sizeof(float) * b.n, hipMemcpyDeviceToHost, compute_));
      KCTC_HIP_CHECK(hipStreamSynchronize(compute_));
      fn_(host_, b.n, user_);
      KCTC_HIP_CHECK(hipMemcpyAsync(b.grad, host_, sizeof(float) * b.n, hipMemcpyHostToDevice, compute_));
      KCTC_HIP_CHECK(hipStreamSynchronize(compute_));
    }
    buckets_.clear();
  }
  int WorldSize() const override { return world_; }
  void AllReduceSum(float *buf, long n, hipStream_t s) override {
    buckets_.push_back({buf, n, s});
    Finish();
  }

 private:
  struct Bucket {
    float *grad;
    long n;
    hipStream_t producer;
  };
  kctc_host_allreduce_fn fn_;
  void *user_;
  int world_;
  hipStream_t compute_;
  hipEvent_t ev_ = nullptr;
  float *host_ = nullptr;
  size_t cap_ = 0;
  std::vector<Bucket> buckets_;
};

// CU-budget probe (kctc_nnet_enable_cu_probe): a one-rank exchange whose
// "all-reduce" of every gradient bucket is a kernel holding `blocks` whole CUs
// for `usec` on the comm stream -- the worst case of an exchange kernel that
// keeps its CUs to itself while the next component's backward recurrence and
// streamed dx GEMM run.  Gated like RcclExchange (the backward stays pinned);
// the gradients are not touched (a sum over one rank).
class CuProbeExchange : public GatedExchange {
 public:
  CuProbeExchange(int blocks, double usec, hipStream_t compute)
      : GatedExchange(compute, blocks), blocks_(blocks), usec_(usec) {}
  int WorldSize() const override { return 1; }
  void AllReduceSum(float *, long, hipStream_t) override {}
  long launches_ = 0;

 protected:
  void Reduce(float *, long) override {
    kctc::cu_hold(comm_stream_, blocks_, usec_);
    launches_++;
  }

 private:
  int blocks_;
  double usec_;
};

}  // namespace

// CUs of the device this process may use: all of them, or its share when
// ranks share a device (kctc_set_cu_partition)
static int g_part = 0, g_nparts = 1;
int kctc_usable_cus_override() {
  if (g_nparts <= 1) return 0;
  int dev = 0, cus = 0;
  KCTC_HIP_CHECK(hipGetDevice(&dev));
  KCTC_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  return cus / g_nparts;
}

void kctc_set_error(const char *msg) { g_err = msg ? msg : ""; }

// the CU mask of share `part` of `nparts`: a contiguous range of mask bits
// (bit b: one CU of XCD b mod 8, scripts/cumask_probe.hip)
static std::vector<uint32_t> partition_mask(int part, int nparts, int cus) {
  const int per = cus / nparts, first = part * per;
  std::vector<uint32_t> mask((cus + 31) / 32, 0u);
  for (int c = first; c < first + per; c++) mask[c / 32] |= 1u << (c % 32);
  return mask;
}

// compute stream at the highest priority (the latency-bound recurrences),
// the weight-gradient side stream at the lowest, and a default-priority
// queue for the streamed GEMMs
void kctcNnetImpl::create_streams() {
  if (g_nparts > 1) {  // ranks sharing the device: this rank's streams on its CU share only
    int cus = 0;
    KCTC_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    const int per = cus / g_nparts;
    const std::vector<uint32_t> mask = partition_mask(g_part, g_nparts, cus);
    KCTC_HIP_CHECK(hipExtStreamCreateWithCUMask(&stream, (uint32_t)mask.size(), mask.data()));
    KCTC_HIP_CHECK(hipExtStreamCreateWithCUMask(&side, (uint32_t)mask.size(), mask.data()));
    KCTC_HIP_CHECK(hipExtStreamCreateWithCUMask(&stream2, (uint32_t)mask.size(), mask.data()));
    kctc::rnn_set_cu_budget(per, kctc::rnn_comm_cus());
    return;
  }
  int lo = 0, hi = 0;
  KCTC_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  KCTC_HIP_CHECK(hipStreamCreateWithPriority(&stream, hipStreamNonBlocking, hi));
  KCTC_HIP_CHECK(hipStreamCreateWithPriority(&side, hipStreamNonBlocking, lo));
  // streamed GEMMs (default priority: a queue of its own, neither the recurrences' nor the side stream's)
  KCTC_HIP_CHECK(hipStreamCreateWithFlags(&stream2, hipStreamNonBlocking));
}

template <typename F>
static int guarded(F f) {
  try {
    f();
    return 0;
  } catch (const std::exception &e) {
    g_err = e.what();
    return 1;
  } catch (...) {
    g_err = "unknown error";
    return 1;
  }
}

static kctc::nnet2::Component &comp(kctcNnet_t n, int c) {
  if (c < 0 || c >= n->nnet.NumComponents()) throw std::out_of_range("component index");
  return n->nnet.GetComponent(c);
}
static kctc::nnet2::UpdatableComponent &ucomp(kctcNnet_t n, int c) {
  auto &x = comp(n, c);
  if (!x.IsUpdatable()) throw std::invalid_argument("component is not updatable");
  return static_cast<kctc::nnet2::UpdatableComponent &>(x);
}

extern "C" {

const char *kctc_last_error(void) { return g_err.c_str(); }

int kctc_nnet_create(kctcNnet_t *out, const char *config, unsigned long long seed, int device) {
  return guarded([&] {
    auto *n = new kctcNnetImpl;
    try {
      n->device = device;
      KCTC_HIP_CHECK(hipSetDevice(device));
      n->create_streams();
      n->activate();
      kctc::nnet2::Rng rng(seed);
      n->nnet.Init(config ? config : "", rng);
    } catch (...) {
      delete n;
      throw;
    }
    *out = n;
  });
}

int kctc_nnet_destroy(kctcNnet_t n) {
  return guarded([&] {
    if (n) {
      n->activate();
      KCTC_HIP_CHECK(hipStreamSynchronize(n->stream));
    }
    delete n;
  });
}

int kctc_nnet_num_components(kctcNnet_t n) { return n ? n->nnet.NumComponents() : -1; }

int kctc_nnet_context(kctcNnet_t n, int *left, int *right) {
  return guarded([&] {
    KCTC_REQUIRE(n && left && right, "kctc_nnet_context: null argument");
    *left = n->nnet.LeftContext();
    *right = n->nnet.RightContext();
  });
}

int kctc_nnet_component_info(kctcNnet_t n, int c, char *buf, size_t len) {
  return guarded([&] {
    n->activate();
    std::string s = comp(n, c).Info();
    if (len) {
      strncpy(buf, s.c_str(), len - 1);
      buf[len - 1] = 0;
    }
  });
}

long kctc_nnet_num_params(kctcNnet_t n, int c) {
  if (!n || c < 0 || c >= n->nnet.NumComponents() || !n->nnet.GetComponent(c).IsUpdatable()) return 0;
  return static_cast<kctc::nnet2::UpdatableComponent &>(n->nnet.GetComponent(c)).NumParameters();
}

int kctc_nnet_get_params(kctcNnet_t n, int c, float *host, long len) {
  return guarded([&] {
    n->activate();
    auto &u = ucomp(n, c);
    if (len != u.NumParameters()) throw std::invalid_argument("size mismatch");
    u.Vectorize(host);
  });
}

int kctc_nnet_set_params(kctcNnet_t n, int c, const float *host, long len) {
  return guarded([&] {
    n->activate();
    auto &u = ucomp(n, c);
    if (len != u.NumParameters()) throw std::invalid_argument("size mismatch");
    u.UnVectorize(host);
  });
}

int kctc_nnet_get_grad(kctcNnet_t n, int c, float *host, long len) {
  return guarded([&] {
    n->activate();
    auto &u = ucomp(n, c);
    if (len != u.NumParameters()) throw std::invalid_argument("size mismatch");
    KCTC_HIP_CHECK(hipStreamSynchronize(n->stream));
    KCTC_HIP_CHECK(hipStreamSynchronize(u.GradStream()));
    KCTC_HIP_CHECK(hipMemcpy(host, u.GradData(), sizeof(float) * len, hipMemcpyDeviceToHost));
  });
}

int kctc_nnet_set_learning_rate(kctcNnet_t n, float lr) {
  return guarded([&] { n->nnet.SetLearningRate(lr); });
}

int kctc_nnet_clip_stats(kctcNnet_t n, int c, double *num_clipped, double *count) {
  return guarded([&] {
    n->activate();
    auto *cg = dynamic_cast<kctc::nnet2::ClipGradientComponent *>(&comp(n, c));
    if (!cg) throw std::invalid_argument("not a ClipGradientComponent");
    cg->SyncStats();
    *num_clipped = cg->NumClipped();
    *count = cg->Count();
  });
}

int kctc_nnet_srand(kctcNnet_t n, unsigned seed) {
  return guarded([&] {
    KCTC_REQUIRE(n, "null nnet");
    n->trainer.Srand(seed);
  });
}

int kctc_nnet_rand_calls(kctcNnet_t n, long *calls) {
  return guarded([&] {
    KCTC_REQUIRE(n && calls, "null argument");
    *calls = n->trainer.RandCalls();
  });
}

int kctc_nnet_last_best_path(kctcNnet_t n, int *ids, long len) {
  return guarded([&] {
    KCTC_REQUIRE(n && ids, "null argument");
    const auto &v = n->trainer.LastBestPath();
    KCTC_REQUIRE(len == (long)v.size(), "kctc_nnet_last_best_path: len != T_max*N of the last minibatch");
    std::copy(v.begin(), v.end(), ids);
  });
}

int kctc_nnet_last_costs(kctcNnet_t n, double *costs, int N) {
  return guarded([&] {
    KCTC_REQUIRE(n && costs, "null argument");
    const auto &v = n->trainer.LastCosts();
    KCTC_REQUIRE(N == (int)v.size(), "kctc_nnet_last_costs: N != minibatch of the last minibatch");
    std::copy(v.begin(), v.end(), costs);
  });
}

int kctc_nnet_last_output(kctcNnet_t n, float *host, long len) {
  return guarded([&] {
    KCTC_REQUIRE(n && host, "null argument");
    n->activate();
    const auto &o = n->trainer.Output();
    KCTC_REQUIRE(o.Data() && len == o.NumRows() * (long)o.NumCols(),
                 "kctc_nnet_last_output: len != T_max*N*A of the last minibatch");
    KCTC_HIP_CHECK(hipStreamSynchronize(n->stream));
    KCTC_HIP_CHECK(hipMemcpy(host, o.Data(), sizeof(float) * len, hipMemcpyDeviceToHost));
  });
}

int kctc_nnet_train_step(kctcNnet_t n, const float *feats_dev, int T_max, int N,
                         const int *num_frames, const int *flat_labels, const int *label_lengths,
                         double *tot_objf, double *tot_accuracy, double *tot_weight) {
  return guarded([&] {
    n->activate();
    auto st = n->trainer.ComputeForMinibatch(feats_dev, T_max, N, num_frames, flat_labels,
                                             label_lengths);
    if (tot_objf) *tot_objf = st.tot_objf;
    if (tot_accuracy) *tot_accuracy = st.tot_accuracy;
    if (tot_weight) *tot_weight = st.tot_weight;
  });
}

int kctc_nnet_train_step_async(kctcNnet_t n, const float *feats_dev, int T_max, int N,
                               const int *num_frames, const int *flat_labels, const int *label_lengths,
                               int *have_stats, double *tot_objf, double *tot_accuracy, double *tot_weight) {
  return guarded([&] {
    n->activate();
    if (have_stats) *have_stats = 0;
    n->trainer.Enqueue(feats_dev, T_max, N, num_frames, flat_labels, label_lengths);
    if (n->trainer.Pending() == 2) {
      auto st = n->trainer.Finish();
      if (have_stats) *have_stats = 1;
      if (tot_objf) *tot_objf = st.tot_objf;
      if (tot_accuracy) *tot_accuracy = st.tot_accuracy;
      if (tot_weight) *tot_weight = st.tot_weight;
    }
  });
}

int kctc_nnet_train_flush(kctcNnet_t n, int *have_stats, double *tot_objf, double *tot_accuracy,
                          double *tot_weight) {
  return guarded([&] {
    n->activate();
    if (have_stats) *have_stats = 0;
    if (n->trainer.Pending()) {
      auto st = n->trainer.Finish();
      if (have_stats) *have_stats = 1;
      if (tot_objf) *tot_objf = st.tot_objf;
      if (tot_accuracy) *tot_accuracy = st.tot_accuracy;
      if (tot_weight) *tot_weight = st.tot_weight;
    }
  });
}

int kctc_nnet_compute_objf(kctcNnet_t n, const float *feats_dev, int T_max, int N,
                           const int *num_frames, const int *flat_labels, const int *label_lengths,
                           double *tot_objf, double *tot_accuracy, double *tot_weight) {
  return guarded([&] {
    n->activate();
    auto st = n->evaluator.ComputeForMinibatch(feats_dev, T_max, N, num_frames, flat_labels,
                                               label_lengths);
    if (tot_objf) *tot_objf = st.tot_objf;
    if (tot_accuracy) *tot_accuracy = st.tot_accuracy;
    if (tot_weight) *tot_weight = st.tot_weight;
  });
}

struct ihipStream_t *kctc_nnet_stream(kctcNnet_t n) { return n ? n->stream : nullptr; }

int kctc_nnet_set_profiling(kctcNnet_t n, int on) {
  return guarded([&] {
    n->activate();
    auto &d = CuDevice::Instantiate();
    d.profiling = on != 0;
    d.prof.clear();
  });
}

int kctc_nnet_profile(kctcNnet_t n, const char *family, double *ms_total, int *launches) {
  return guarded([&] {
    auto &d = CuDevice::Instantiate();
    auto it = d.prof.find(family ? family : "");
    *ms_total = it == d.prof.end() ? 0.0 : it->second.first;
    *launches = it == d.prof.end() ? 0 : it->second.second;
  });
}

int kctc_nnet_write(kctcNnet_t n, const char *path) { return kctc_nnet_write_kaldi(n, path, 0); }

int kctc_nnet_write_kaldi(kctcNnet_t n, const char *path, int binary) {
  return guarded([&] {
    n->activate();
    std::ofstream os(path, std::ios::binary | std::ios::trunc);
    if (!os) throw std::runtime_error(std::string("cannot open ") + path);
    kctc::kio::InitOutput(os, binary != 0);
    n->nnet.Write(os, binary != 0);
    if (!os) throw std::runtime_error(std::string("write failed: ") + path);
  });
}

static std::string slurp(const char *path) {
  std::ifstream is(path, std::ios::binary);
  if (!is) throw std::runtime_error(std::string("cannot open ") + path);
  std::ostringstream ss;
  ss << is.rdbuf();
  return ss.str();
}

static kctcNnetImpl *new_on_device(int device) {
  auto *n = new kctcNnetImpl;
  try {
    n->device = device;
    KCTC_HIP_CHECK(hipSetDevice(device));
    n->create_streams();
    n->activate();
  } catch (...) {
    delete n;
    throw;
  }
  return n;
}

// whole file in memory (models are ~0.1 GB); `am`: the nnet2-ctc model form
// (CtcTransitionModel + Nnet + priors, nnet2-ctc-train-simple.cc:58-64)
static void read_model(kctcNnetImpl *n, const char *path, bool am) {
  std::istringstream is(slurp(path));
  const bool binary = kctc::kio::InitInput(is);
  if (am && kctc::kio::PeekToken(is, binary) == "<TransitionModel>") {
    // kept opaque: everything up to and including the "</TransitionModel> " token
    const std::string &buf = is.str();
    const std::string end_tok = "</TransitionModel> ";
    const auto start = (size_t)is.tellg();
    const auto e = buf.find(end_tok, start);
    if (e == std::string::npos) throw std::runtime_error("unterminated <TransitionModel>");
    // text mode: TransitionModel::Write ends the token with a newline
    // (src/hmm/transition-model.cc:316-317); keep it, so write-back is byte-identical
    size_t stop = e + end_tok.size();
    if (!binary && stop < buf.size() && buf[stop] == '\n') stop++;
    n->trans_model = buf.substr(start, stop - start);
    n->trans_model_binary = binary;
    is.seekg((std::streamoff)stop);
  }
  n->nnet.Read(is, binary);
  if (am) {
    n->priors = kctc::kio::ReadFloatVector(is, binary);
    if (!n->priors.empty() && (int)n->priors.size() != n->nnet.OutputDim())
      throw std::runtime_error("AmNnet priors dimension != network output dimension");
  }
}

int kctc_nnet_read(kctcNnet_t *out, const char *path, int device) {
  return guarded([&] {
    auto *n = new_on_device(device);
    try {
      read_model(n, path, false);
    } catch (...) {
      delete n;
      throw;
    }
    *out = n;
  });
}

int kctc_am_nnet_read(kctcNnet_t *out, const char *path, int device) {
  return guarded([&] {
    auto *n = new_on_device(device);
    try {
      read_model(n, path, true);
    } catch (...) {
      delete n;
      throw;
    }
    *out = n;
  });
}

int kctc_am_nnet_write(kctcNnet_t n, const char *path, int binary) {
  return guarded([&] {
    n->activate();
    if (!n->trans_model.empty() && n->trans_model_binary != (binary != 0))
      throw std::runtime_error("the transition model was read in the other mode; write the model in that mode");
    std::ofstream os(path, std::ios::binary | std::ios::trunc);
    if (!os) throw std::runtime_error(std::string("cannot open ") + path);
    kctc::kio::InitOutput(os, binary != 0);
    os.write(n->trans_model.data(), (std::streamsize)n->trans_model.size());
    n->nnet.Write(os, binary != 0);
    kctc::kio::WriteFloatVector(os, binary != 0, n->priors.data(), (long)n->priors.size());
    if (!os) throw std::runtime_error(std::string("write failed: ") + path);
  });
}

int kctc_am_nnet_num_priors(kctcNnet_t n) { return n ? (int)n->priors.size() : -1; }

int kctc_am_nnet_get_priors(kctcNnet_t n, float *priors, int dim) {
  return guarded([&] {
    KCTC_REQUIRE(dim == (int)n->priors.size() && (dim == 0 || priors), "kctc_am_nnet_get_priors: bad size");
    std::copy(n->priors.begin(), n->priors.end(), priors);
  });
}

int kctc_am_nnet_set_priors(kctcNnet_t n, const float *priors, int dim) {
  return guarded([&] {  // AmNnet::SetPriors (am-nnet.cc:44-55)
    const int pdfs = n->nnet.OutputDim();
    KCTC_REQUIRE(dim >= 0 && dim <= pdfs, "Dimension of priors cannot exceed number of pdfs.");
    KCTC_REQUIRE(dim == 0 || priors, "kctc_am_nnet_set_priors: null priors");
    n->priors.assign(priors, priors + dim);
    if (dim > 0 && dim < pdfs) n->priors.resize(pdfs, 0.f);
  });
}

int kctc_dp_unique_id(void *uid128) {
  return guarded([&] {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) throw std::runtime_error("ncclGetUniqueId failed");
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    memcpy(uid128, &id, sizeof(id));
  });
}

int kctc_nnet_enable_dp(kctcNnet_t n, const void *uid128, int rank, int world_size) {
  return guarded([&] {
    n->activate();
    KCTC_REQUIRE(world_size >= 0 && (world_size == 0 || (rank >= 0 && rank < world_size && uid128)),
                 "kctc_nnet_enable_dp: bad rank / world size");
    KCTC_REQUIRE(n->trainer.Pending() == 0, "kctc_nnet_enable_dp with minibatches in flight");
    delete n->dp;
    n->dp = nullptr;
    n->trainer.SetExchange(nullptr);
    if (world_size >= 1) {  // one rank included: the same communicator and all-reduce path
      n->dp = new RcclExchange(uid128, rank, world_size, n->stream);
      n->trainer.SetExchange(n->dp_average ? nullptr : n->dp);
    }
  });
}

int kctc_nnet_enable_dp_host(kctcNnet_t n, kctc_host_allreduce_fn fn, void *user, int world_size) {
  return guarded([&] {
    KCTC_REQUIRE(n && fn && world_size >= 1, "kctc_nnet_enable_dp_host: bad argument");
    KCTC_REQUIRE(n->trainer.Pending() == 0, "kctc_nnet_enable_dp_host with minibatches in flight");
    n->activate();
    delete n->dp;
    n->dp = nullptr;
    n->trainer.SetExchange(nullptr);
    n->dp = new HostExchange(fn, user, world_size, n->stream);
    n->trainer.SetExchange(n->dp_average ? nullptr : n->dp);
  });
}

int kctc_nnet_enable_cu_probe(kctcNnet_t n, int blocks, double usec) {
  return guarded([&] {
    KCTC_REQUIRE(n && blocks >= 0 && usec >= 0, "kctc_nnet_enable_cu_probe: bad argument");
    KCTC_REQUIRE(n->trainer.Pending() == 0, "kctc_nnet_enable_cu_probe with minibatches in flight");
    n->activate();
    delete n->dp;
    n->dp = nullptr;
    n->trainer.SetExchange(nullptr);
    if (blocks > 0) {
      n->dp = new CuProbeExchange(blocks, usec, n->stream);
      n->trainer.SetExchange(n->dp);
    }
  });
}

int kctc_set_cu_partition(int part, int nparts) {
  return guarded([&] {
    KCTC_REQUIRE(nparts >= 1 && nparts <= 8 && part >= 0 && part < nparts, "kctc_set_cu_partition: bad partition");
    g_part = part;
    g_nparts = nparts;
    kctc::rnn_set_cu_budget(kctc_usable_cus_override(), kctc::rnn_comm_cus());
  });
}

int kctc_cu_partition_probe(int part, int nparts, unsigned *ids, int max_ids, int *n_ids) {
  return guarded([&] {
    KCTC_REQUIRE(nparts >= 1 && nparts <= 8 && part >= 0 && part < nparts && ids && n_ids && max_ids > 0,
                 "kctc_cu_partition_probe: bad arguments");
    int dev = 0, cus = 0;
    KCTC_HIP_CHECK(hipGetDevice(&dev));
    KCTC_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const std::vector<uint32_t> mask = partition_mask(part, nparts, cus);
    hipStream_t s = nullptr;
    KCTC_HIP_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    const int blocks = 8 * cus;
    unsigned *d = nullptr;
    KCTC_HIP_CHECK(hipMalloc(&d, sizeof(unsigned) * blocks));
    kctc::cu_where(s, d, blocks, 50.0);  // long enough that the blocks spread over every CU of the share
    std::vector<unsigned> h(blocks);
    KCTC_HIP_CHECK(hipMemcpyAsync(h.data(), d, sizeof(unsigned) * blocks, hipMemcpyDeviceToHost, s));
    KCTC_HIP_CHECK(hipStreamSynchronize(s));
    (void)hipFree(d);
    (void)hipStreamDestroy(s);
    std::sort(h.begin(), h.end());
    h.erase(std::unique(h.begin(), h.end()), h.end());
    *n_ids = (int)std::min<size_t>(h.size(), (size_t)max_ids);
    std::copy(h.begin(), h.begin() + *n_ids, ids);
  });
}

int kctc_nnet_inject_step_error(kctcNnet_t n, unsigned word) {
  return guarded([&] {
    KCTC_REQUIRE(n, "null nnet");
    n->trainer.InjectStepError(word);
  });
}

int kctc_nnet_set_dp_mode(kctcNnet_t n, int mode) {
  return guarded([&] {
    KCTC_REQUIRE(n && (mode == 0 || mode == 1), "kctc_nnet_set_dp_mode: mode must be 0 or 1");
    KCTC_REQUIRE(n->trainer.Pending() == 0, "kctc_nnet_set_dp_mode with minibatches in flight");
    n->dp_average = mode == 1;
    n->trainer.SetExchange(n->dp && !n->dp_average ? n->dp : nullptr);
  });
}

// nnet-am-average over the data-parallel ranks (src/nnet2bin/nnet-am-average.cc:
// 185-241 with the default weights 1/num-models), on the component API the tool
// uses: every rank's updatable component is Scale(1/world)d (the tool's scale
// of model 1 by its weight), then the collective sum adds the other ranks'
// scaled copies (the tool's Add(weight, model i)), on the compute stream.
int kctc_nnet_average_params(kctcNnet_t n) {
  return guarded([&] {
    KCTC_REQUIRE(n && n->dp, "kctc_nnet_average_params: data parallelism not enabled");
    KCTC_REQUIRE(n->trainer.Pending() == 0, "kctc_nnet_average_params with minibatches in flight");
    n->activate();
    const int world = n->dp->WorldSize();
    for (int c = 0; c < n->nnet.NumComponents(); c++) {
      auto *u = dynamic_cast<kctc::nnet2::UpdatableComponent *>(&n->nnet.GetComponent(c));
      if (!u) continue;
      if (world > 1) u->Scale(1.f / (float)world);
      n->dp->AllReduceSum(u->ParamData(), u->NumParameters(), n->stream);
    }
    KCTC_HIP_CHECK(hipStreamSynchronize(n->stream));
  });
}

int kctc_nnet_set_precision(kctcNnet_t n, int precision) {
  return guarded([&] {
    KCTC_REQUIRE(n && (precision == 0 || precision == 1), "kctc_nnet_set_precision: precision must be 0 or 1");
    KCTC_REQUIRE(n->trainer.Pending() == 0, "kctc_nnet_set_precision with minibatches in flight");
    for (int c = 0; c < n->nnet.NumComponents(); c++)
      if (auto *r = dynamic_cast<kctc::nnet2::CuDNNRecurrentComponent *>(&n->nnet.GetComponent(c)))
        r->SetPrecision(precision);
  });
}

int kctc_nnet_set_momentum(kctcNnet_t n, float momentum) {
  return guarded([&] {
    KCTC_REQUIRE(n, "null nnet");
    n->activate();
    n->nnet.SetMomentum(momentum);
  });
}

int kctc_nnet_train_simple(kctcNnet_t n, struct kctcEgsReader_ *r, long max_minibatches, long *num_egs,
                           double *tot_weight, double *tot_objf, double *tot_accuracy) {
  return guarded([&] {
    KCTC_REQUIRE(n && r, "kctc_nnet_train_simple: null argument");
    n->activate();
    long egs = 0, mbs = 0;
    double w = 0, objf = 0, acc = 0;
    while (max_minibatches <= 0 || mbs < max_minibatches) {
      std::unique_ptr<kctc::egs::Minibatch> mb = r->r.Next();  // GetNextMinibatch
      if (!mb) break;
      if (mb->InputDim() != n->nnet.InputDim())
        throw std::invalid_argument("egs input dim " + std::to_string(mb->InputDim()) + " != nnet input dim " +
                                    std::to_string(n->nnet.InputDim()));
      if (mb->num_splice != n->nnet.NumSplice())
        throw std::invalid_argument("the egs reader was opened with a context other than the network's "
                                    "(kctc_nnet_context)");
      n->egs_feats.ensure(sizeof(float) * (size_t)mb->T_max * mb->N * mb->num_splice * mb->InputDim());
      n->egs_scratch.ensure(kctc::egs::format_scratch_bytes(*mb));
      kctc::egs::format_on_device(*mb, n->egs_feats.f(), n->egs_scratch.p, n->egs_scratch.bytes, n->stream);
      const auto st = n->trainer.ComputeForMinibatch(n->egs_feats.f(), mb->T_max, mb->N, mb->num_frames.data(),
                                                     mb->labels.data(), mb->label_lengths.data());
      objf += st.tot_objf;
      acc += st.tot_accuracy;
      w += st.tot_weight;
      egs += mb->N;
      mbs++;
    }
    if (num_egs) *num_egs = egs;
    if (tot_weight) *tot_weight = w;
    if (tot_objf) *tot_objf = objf;
    if (tot_accuracy) *tot_accuracy = acc;
  });
}

size_t kctc_ctc_decodable_scratch_bytes(int T) { return kctc::ctc_decodable_scratch_bytes(T > 0 ? T : 1) + 256; }

int kctc_softmax_rows(struct ihipStream_t *stream, const float *in, long rows, int cols, float *out) {
  return guarded([&] {
    KCTC_REQUIRE(in && out && rows >= 0 && cols > 0, "kctc_softmax_rows: bad argument");
    kctc::softmax_rows(stream, in, rows, cols, out);
    KCTC_HIP_CHECK(hipGetLastError());
  });
}

int kctc_ctc_decodable(struct ihipStream_t *stream, const float *probs, int T, int A, const float *priors,
                       float prob_scale, float blank_threshold, float floor_value, float *out, void *scratch,
                       int *num_kept) {
  return guarded([&] {
    KCTC_REQUIRE(probs && out && scratch && num_kept && T > 0 && A > 0, "kctc_ctc_decodable: bad argument");
    int *kept_dev = reinterpret_cast<int *>(static_cast<char *>(scratch) + kctc::ctc_decodable_scratch_bytes(T));
    kctc::ctc_decodable(stream, probs, T, A, priors, prob_scale, blank_threshold, floor_value, out, scratch,
                        kept_dev);
    KCTC_HIP_CHECK(hipGetLastError());
    KCTC_HIP_CHECK(hipMemcpyAsync(num_kept, kept_dev, sizeof(int), hipMemcpyDeviceToHost, stream));
    KCTC_HIP_CHECK(hipStreamSynchronize(stream));
  });
}

int kctc_nnet_propagate(kctcNnet_t n, const float *feats_dev, int T_max, int N, float *out_dev, long len) {
  return guarded([&] {
    KCTC_REQUIRE(n && feats_dev && out_dev, "kctc_nnet_propagate: null argument");
    n->activate();
    const auto &o = n->evaluator.Forward(feats_dev, T_max, N);
    KCTC_REQUIRE(len == o.NumRows() * (long)o.NumCols(), "kctc_nnet_propagate: len != T_max*N*output_dim");
    KCTC_HIP_CHECK(hipMemcpyAsync(out_dev, o.Data(), sizeof(float) * len, hipMemcpyDeviceToDevice, n->stream));
    KCTC_HIP_CHECK(hipStreamSynchronize(n->stream));
  });
}

int kctc_am_nnet_decodable(kctcNnet_t n, const float *feats_dev, int T, float prob_scale, float blank_threshold,
                           float *out_host, int *num_rows) {
  return guarded([&] {
    KCTC_REQUIRE(n && feats_dev && out_host && num_rows && T > 0, "kctc_am_nnet_decodable: bad argument");
    n->activate();
    // NnetComputation(nnet, feats, pad_input = true) (ctc-decodable-am-nnet.cc:28-52,
    // nnet-compute.cc:64-90): T output frames from the T feature rows, the
    // first / last frame repeated LeftContext / RightContext times; a spliced
    // network reads num_splice rows per output frame (FormatNnetInput layout)
    const float *in = feats_dev;
    const int ns = n->nnet.NumSplice();
    if (ns > 1) {
      n->dec_input.ensure(sizeof(float) * (size_t)T * ns * n->nnet.InputDim());
      kctc::pad_splice_input(n->stream, feats_dev, T, n->nnet.InputDim(), n->nnet.LeftContext(), ns,
                             n->dec_input.f());
      in = n->dec_input.f();
    }
    const auto &o = n->evaluator.Forward(in, T, 1);
    const int A = o.NumCols();
    auto &out = n->dec_out, &scratch = n->dec_scratch;
    const float *pd = nullptr;
    if (!n->priors.empty()) {
      KCTC_REQUIRE((int)n->priors.size() == A, "priors dimension != network output dimension");
      if (n->dec_priors_host != n->priors) {
        n->dec_priors.ensure(sizeof(float) * A);
        KCTC_HIP_CHECK(hipMemcpyAsync(n->dec_priors.p, n->priors.data(), sizeof(float) * A, hipMemcpyHostToDevice,
                                      n->stream));
        KCTC_HIP_CHECK(hipStreamSynchronize(n->stream));  // the source is the host vector
        n->dec_priors_host = n->priors;
      }
      pd = n->dec_priors.f();
    }
    out.ensure(sizeof(float) * (size_t)T * A);
    scratch.ensure(kctc_ctc_decodable_scratch_bytes(T));
    int kept = 0;
    const int st = kctc_ctc_decodable(n->stream, o.Data(), T, A, pd, prob_scale, blank_threshold, 1.0e-10f, out.f(),
                                      scratch.p, &kept);
    if (st) throw std::runtime_error(g_err);
    KCTC_HIP_CHECK(hipStreamSynchronize(n->stream));
    KCTC_HIP_CHECK(hipMemcpy(out_host, out.p, sizeof(float) * (size_t)kept * A, hipMemcpyDeviceToHost));
    *num_rows = kept;
  });
}

int kctc_nnet_compute_prob(kctcNnet_t n, const char *rspecifier, long *num_examples, double *tot_like,
                           double *tot_accuracy, double *tot_weight) {
  return guarded([&] {
    KCTC_REQUIRE(n && rspecifier, "kctc_nnet_compute_prob: null argument");
    n->activate();
    kctc::egs::ArchiveReader reader(rspecifier);
    std::vector<kctc::egs::Example> batch;
    long ne = 0;
    double like = 0, acc = 0, w = 0;
    auto run = [&]() {  // ComputeNnetObjf on one batch (ctc-nnet-update.cc:426-431)
      std::unique_ptr<kctc::egs::Minibatch> mb =
          kctc::egs::pack_minibatch(batch, n->nnet.LeftContext(), n->nnet.RightContext());
      if (mb->InputDim() != n->nnet.InputDim())
        throw std::invalid_argument("egs input dim " + std::to_string(mb->InputDim()) + " != nnet input dim " +
                                    std::to_string(n->nnet.InputDim()));
      n->egs_feats.ensure(sizeof(float) * (size_t)mb->T_max * mb->N * mb->num_splice * mb->InputDim());
      n->egs_scratch.ensure(kctc::egs::format_scratch_bytes(*mb));
      kctc::egs::format_on_device(*mb, n->egs_feats.f(), n->egs_scratch.p, n->egs_scratch.bytes, n->stream);
      const auto st = n->evaluator.ComputeForMinibatch(n->egs_feats.f(), mb->T_max, mb->N, mb->num_frames.data(),
                                                       mb->labels.data(), mb->label_lengths.data());
      like += st.tot_objf;
      acc += st.tot_accuracy;
      w += st.tot_weight;  // TotalNnetTrainingWeight: sum of label counts
      batch.clear();
    };
    kctc::egs::Example eg;
    while (reader.Next(&eg)) {
      if (batch.size() == 10) run();
      batch.push_back(std::move(eg));
      eg = kctc::egs::Example();
      ne++;
    }
    if (!batch.empty()) run();
    if (num_examples) *num_examples = ne;
    if (tot_like) *tot_like = like;
    if (tot_accuracy) *tot_accuracy = acc;
    if (tot_weight) *tot_weight = w;
  });
}

int kctc_levenshtein(const int *ref, int nref, const int *hyp, int nhyp) {
  if ((nref > 0 && !ref) || (nhyp > 0 && !hyp)) return -1;
  return kctc::nnet2::levenshtein(ref, nref, hyp, nhyp);
}

int kctc_format_input(const float *feats, const int *num_frames, int N, int dim, int T_max,
                      float *out) {
  return guarded([&] {
    // FormatNnetInput (ctc-nnet-update.cc:351-424): row t*N+n, zero padded
    memset(out, 0, sizeof(float) * (size_t)T_max * N * dim);
    long off = 0;
    for (int n = 0; n < N; n++) {
      if (num_frames[n] > T_max) throw std::invalid_argument("num_frames > T_max");
      for (int t = 0; t < num_frames[n]; t++)
        memcpy(out + ((size_t)t * N + n) * dim, feats + (off + t) * (size_t)dim, sizeof(float) * dim);
      off += num_frames[n];
    }
  });
}

long kctc_synth_minibatch(unsigned long long seed, int T_max, int N, int dim, int A,
                          double label_ratio, float *feats, int *num_frames, int *flat_labels,
                          int *label_lengths) {
  kctc::nnet2::Rng rng(seed);
  long nl = 0;
  for (int n = 0; n < N; n++) {
    int T = n == 0 ? T_max : T_max - (int)std::floor(rng.uniform() * 0.1 * T_max);
    if (T < 1) T = 1;
    num_frames[n] = T;
    long L = (long)std::floor(T * label_ratio);
    L = std::min<long>(L, 639);
    L = std::min<long>(L, (T - 1) / 2);
    L = std::max<long>(L, 0);
    label_lengths[n] = (int)L;
    int prev = -1;
    for (long i = 0; i < L; i++) {
      int v;
      do {
        v = 1 + (int)(rng.next() % (unsigned long long)(A - 1));
      } while (v == prev && A > 2);
      flat_labels[nl++] = v;
      prev = v;
    }
  }
  if (feats) {
    for (int t = 0; t < T_max; t++)
      for (int n = 0; n < N; n++) {
        float *row = feats + ((size_t)t * N + n) * dim;
        if (t < num_frames[n])
          for (int j = 0; j < dim; j++) row[j] = (float)rng.gauss();
        else
          memset(row, 0, sizeof(float) * dim);
      }
  }
  return nl;
}

}  // extern "C"
