// component_api.cpp -- C ABI of include/kaldi_nnet2_component.h: standalone
// nnet2 components (the Component plug-in point, nnet-component.h:157-348)
// and the nnet-am-average component loops.
#include "kaldi_nnet2_component.h"
#include "test_hooks.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "common.h"
#include "kaldi_io.h"
#include "nnet.h"
#include "nnet_handle.h"

using kctc::nnet2::ChunkInfo;
using kctc::nnet2::ClipGradientComponent;
using kctc::nnet2::Component;
using kctc::nnet2::CuDevice;
using kctc::nnet2::CuMatrixBase;
using kctc::nnet2::CuDNNRecurrentComponent;
using kctc::nnet2::SoftmaxComponent;
using kctc::nnet2::UpdatableComponent;

struct kctcComponentImpl {
  int device = 0;
  hipStream_t stream = nullptr;
  // test hook (kctc_test_component_side_streams): the trainer's side and
  // dx-stream queues, so that the component streams and prepacks as in training
  hipStream_t side = nullptr, stream2 = nullptr;
  std::unique_ptr<Component> c;
  kctc::GlibcRand rng{0};  // ClipGradient self-repair draws (srand(0))
  explicit kctcComponentImpl(int dev) : device(dev) {
    KCTC_HIP_CHECK(hipSetDevice(dev));
    KCTC_HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  }
  ~kctcComponentImpl() {
    if (stream) {
      (void)hipStreamSynchronize(stream);
      auto &d = CuDevice::Instantiate();
      if (d.stream == stream) d.stream = nullptr;
    }
    c.reset();
    for (hipStream_t s2 : {side, stream2})
      if (s2) {
        (void)hipStreamSynchronize(s2);
        auto &d = CuDevice::Instantiate();
        if (d.side == s2) d.side = nullptr;
        if (d.stream2 == s2) d.stream2 = nullptr;
        (void)hipStreamDestroy(s2);
      }
    if (stream) (void)hipStreamDestroy(stream);
  }
  // everything of a standalone component on its one stream (no side streams
  // unless the test hook gave it the trainer's two)
  void activate() {
    KCTC_HIP_CHECK(hipSetDevice(device));
    auto &d = CuDevice::Instantiate();
    d.device = device;
    d.stream = stream;
    d.side = side;
    d.stream2 = stream2;
  }
  void sync() {
    for (hipStream_t s2 : {side, stream2})
      if (s2) KCTC_HIP_CHECK(hipStreamSynchronize(s2));
    KCTC_HIP_CHECK(hipStreamSynchronize(stream));
  }
  UpdatableComponent &u() {
    if (!c->IsUpdatable()) throw std::invalid_argument(c->Type() + " is not an UpdatableComponent");
    return static_cast<UpdatableComponent &>(*c);
  }
};

namespace {

std::string slurp(const char *path) {
  std::ifstream is(path, std::ios::binary);
  if (!is) throw std::runtime_error(std::string("cannot open ") + path);
  std::ostringstream ss;
  ss << is.rdbuf();
  return ss.str();
}

// input rows per output frame: the span of Context() (SpliceComponent)
int num_splice(const Component &c) {
  const std::vector<int> ctx = c.Context();
  return ctx.back() - ctx.front() + 1;
}

// ChunkInfo pair of a T x N time-major block (Nnet::ComputeChunkInfo for one
// component, contiguous case): the output frame sits -Context().front()
// frames after the chunk's first input row
void chunk_infos(const Component &c, int T, int N, ChunkInfo *in, ChunkInfo *out) {
  in->feat_dim = c.InputDim();
  in->num_chunks = N;
  in->chunk_size = T;
  in->first_offset = 0;
  *out = *in;
  out->feat_dim = c.OutputDim();
  out->first_offset = -c.Context().front();
}

void set_minibatch(Component &c, int N) {
  if (auto *r = dynamic_cast<CuDNNRecurrentComponent *>(&c)) r->SetMiniBatch(N);
}

kctcComponentImpl *wrap(Component *c, int device) {
  std::unique_ptr<Component> own(c);
  auto *h = new kctcComponentImpl(device);
  h->c = std::move(own);
  return h;
}

// Scale / Add of the component kinds nnet-am-average touches: UpdatableComponent
// and the NonlinearComponent statistics (SoftmaxComponent here); ClipGradient
// counters have the same pair in the reference (nnet-cudnn-component.cc:1064-1073)
void scale_component(Component &c, float s) {
  if (c.IsUpdatable()) static_cast<UpdatableComponent &>(c).Scale(s);
  else if (auto *sm = dynamic_cast<SoftmaxComponent *>(&c)) sm->Scale(s);
  else if (auto *cg = dynamic_cast<ClipGradientComponent *>(&c)) cg->Scale(s);
  else throw std::invalid_argument(c.Type() + " has no Scale()");
}
void add_component(Component &c, float alpha, const Component &o) {
  if (c.Type() != o.Type()) throw std::invalid_argument("Add: components of different type");
  if (c.IsUpdatable())
    static_cast<UpdatableComponent &>(c).Add(alpha, static_cast<const UpdatableComponent &>(o));
  else if (auto *sm = dynamic_cast<SoftmaxComponent *>(&c))
    sm->Add(alpha, static_cast<const SoftmaxComponent &>(o));
  else if (auto *cg = dynamic_cast<ClipGradientComponent *>(&c))
    cg->Add(alpha, static_cast<const ClipGradientComponent &>(o));
  else
    throw std::invalid_argument(c.Type() + " has no Add()");
}

int average_end(const kctc::nnet2::Nnet &n, bool skip_last) {
  if (!skip_last) return n.NumComponents();
  const int e = n.LastUpdatableComponent();
  if (e < 0) throw std::invalid_argument("Network has no updatable components.");
  return e;
}

// the nnet-am-average loops: UpdatableComponent and NonlinearComponent only
bool averaged(const Component &c) { return c.IsUpdatable() || dynamic_cast<const SoftmaxComponent *>(&c); }

void nnet_scale(kctcNnetImpl *n, float s, bool skip_last) {
  const int end = average_end(n->nnet, skip_last);
  for (int c = 0; c < end; c++)
    if (averaged(n->nnet.GetComponent(c))) scale_component(n->nnet.GetComponent(c), s);
}
void nnet_add(kctcNnetImpl *n, float alpha, kctcNnetImpl *o, bool skip_last) {
  if (o->nnet.NumComponents() != n->nnet.NumComponents())
    throw std::invalid_argument("Networks must have the same structure.");
  const int end = average_end(n->nnet, skip_last);
  KCTC_HIP_CHECK(hipStreamSynchronize(o->stream));  // the other's parameters are complete
  for (int c = 0; c < end; c++) {
    auto &a = n->nnet.GetComponent(c);
    if (averaged(a)) add_component(a, alpha, o->nnet.GetComponent(c));
  }
}

}  // namespace

extern "C" {

int kctc_component_init(kctcComponent_t *out, const char *line, unsigned long long seed, int device) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(out && line, "kctc_component_init: null argument");
    std::istringstream is(line);
    std::string type, rest, tok;
    is >> type;
    while (is >> tok) rest += (rest.empty() ? "" : " ") + tok;
    Component *c = Component::NewComponentOfType(type);
    if (!c) throw std::invalid_argument("Unknown component type " + type);
    std::unique_ptr<kctcComponentImpl> h(wrap(c, device));
    h->activate();
    kctc::nnet2::Rng rng(seed);
    h->c->InitFromString(rest, rng);
    h->sync();
    *out = h.release();
  });
}

int kctc_component_read(kctcComponent_t *out, const char *path, int device) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(out && path, "kctc_component_read: null argument");
    std::unique_ptr<kctcComponentImpl> h(new kctcComponentImpl(device));
    h->activate();
    std::istringstream is(slurp(path));
    const bool binary = kctc::kio::InitInput(is);
    h->c.reset(Component::ReadNew(is, binary));
    h->sync();
    *out = h.release();
  });
}

int kctc_component_write(kctcComponent_t h, const char *path, int binary) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h && path, "kctc_component_write: null argument");
    h->activate();
    std::ofstream os(path, std::ios::binary | std::ios::trunc);
    if (!os) throw std::runtime_error(std::string("cannot open ") + path);
    kctc::kio::InitOutput(os, binary != 0);
    h->c->Write(os, binary != 0);
    if (!os) throw std::runtime_error(std::string("write failed: ") + path);
  });
}

int kctc_component_copy(kctcComponent_t h, kctcComponent_t *out) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h && out, "kctc_component_copy: null argument");
    h->activate();
    Component *c = h->c->Copy();
    h->sync();  // the copy's device buffers were written on h's stream
    *out = wrap(c, h->device);
  });
}

int kctc_component_destroy(kctcComponent_t h) {
  return kctc_guarded([&] {
    if (h) h->activate();
    delete h;
  });
}

static void put_string(const std::string &s, char *buf, size_t len) {
  KCTC_REQUIRE(buf || !len, "null buffer");
  if (len) {
    strncpy(buf, s.c_str(), len - 1);
    buf[len - 1] = 0;
  }
}

int kctc_component_type(kctcComponent_t h, char *buf, size_t len) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h, "null component");
    put_string(h->c->Type(), buf, len);
  });
}

int kctc_component_info(kctcComponent_t h, char *buf, size_t len) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h, "null component");
    h->activate();
    put_string(h->c->Info(), buf, len);
  });
}

int kctc_component_dims(kctcComponent_t h, int *in, int *out) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h && in && out, "kctc_component_dims: null argument");
    *in = h->c->InputDim();
    *out = h->c->OutputDim();
  });
}

int kctc_component_context(kctcComponent_t h, int *offsets, int cap, int *n) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h && n && (offsets || cap <= 0), "kctc_component_context: null argument");
    const std::vector<int> ctx = h->c->Context();
    *n = (int)ctx.size();
    for (int i = 0; i < (int)ctx.size() && i < cap; i++) offsets[i] = ctx[i];
  });
}

int kctc_component_backprop_needs(kctcComponent_t h, int *needs_input, int *needs_output) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h && needs_input && needs_output, "null argument");
    *needs_input = h->c->BackpropNeedsInput() ? 1 : 0;
    *needs_output = h->c->BackpropNeedsOutput() ? 1 : 0;
  });
}

int kctc_component_is_updatable(kctcComponent_t h) { return h && h->c->IsUpdatable() ? 1 : 0; }

int kctc_component_propagate(kctcComponent_t h, int T, int N, const float *in, long in_len, float *out,
                             long out_len) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h && in && out && T > 0 && N > 0, "kctc_component_propagate: bad argument");
    Component &c = *h->c;
    const long rows = (long)T * N;
    KCTC_REQUIRE(in_len == rows * num_splice(c) * c.InputDim(),
                 "kctc_component_propagate: in_len != T*N*num_splice*InputDim");
    KCTC_REQUIRE(out_len == rows * c.OutputDim(), "kctc_component_propagate: out_len != T*N*OutputDim");
    h->activate();
    set_minibatch(c, N);
    ChunkInfo ii, oi;
    chunk_infos(c, T, N, &ii, &oi);
    const CuMatrixBase x(const_cast<float *>(in), rows * num_splice(c), c.InputDim());
    CuMatrixBase y(out, rows, c.OutputDim());
    c.Propagate(ii, oi, x, &y);
    h->sync();
  });
}

int kctc_component_backprop(kctcComponent_t h, int T, int N, const float *in_value, long in_len,
                            const float *out_value, long out_len, const float *out_deriv, long od_len,
                            kctcComponent_t to_update, float *in_deriv, long id_len) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h && out_deriv && T > 0 && N > 0, "kctc_component_backprop: bad argument");
    Component &c = *h->c;
    const long rows = (long)T * N, in_rows = rows * num_splice(c);
    KCTC_REQUIRE(!c.BackpropNeedsInput() || (in_value && in_len == in_rows * c.InputDim()),
                 "kctc_component_backprop: in_value missing or in_len != T*N*num_splice*InputDim");
    KCTC_REQUIRE(!c.BackpropNeedsOutput() || (out_value && out_len == rows * c.OutputDim()),
                 "kctc_component_backprop: out_value missing or out_len != T*N*OutputDim");
    KCTC_REQUIRE(od_len == rows * c.OutputDim(), "kctc_component_backprop: out_deriv_len != T*N*OutputDim");
    KCTC_REQUIRE(!in_deriv || id_len == in_rows * c.InputDim(),
                 "kctc_component_backprop: in_deriv_len != T*N*num_splice*InputDim");
    if (to_update) {
      KCTC_REQUIRE(to_update->c->Type() == c.Type(), "kctc_component_backprop: to_update of another type");
      KCTC_REQUIRE(to_update->device == h->device, "kctc_component_backprop: to_update on another device");
    }
    if (auto *r = dynamic_cast<CuDNNRecurrentComponent *>(&c))
      KCTC_REQUIRE(r->PropagatedShape(T, N),
                   "CuDNNRecurrentComponent::Backprop needs a Propagate of this component on the same T x N "
                   "input first (cuDNN's reserve-space contract)");
    if (to_update) KCTC_HIP_CHECK(hipStreamSynchronize(to_update->stream));
    h->activate();
    ChunkInfo ii, oi;
    chunk_infos(c, T, N, &ii, &oi);
    const CuMatrixBase x(const_cast<float *>(in_value), in_value ? in_rows : 0, c.InputDim());
    const CuMatrixBase y(const_cast<float *>(out_value), out_value ? rows : 0, c.OutputDim());
    const CuMatrixBase dy(const_cast<float *>(out_deriv), rows, c.OutputDim());
    CuMatrixBase dx(in_deriv, in_rows, c.InputDim());
    Component *tu = to_update ? to_update->c.get() : nullptr;
    if (auto *cg = dynamic_cast<ClipGradientComponent *>(&c)) cg->rng_ = &h->rng;
    c.Backprop(ii, oi, x, y, dy, tu, in_deriv ? &dx : nullptr);
    CuDevice::Instantiate().Join();  // (the test hook's side stream: the weight GEMMs)
    // the reference updates inside Backprop (CuDNNRecurrentComponent::Update,
    // AffineComponent::UpdateSimple); the mirror defers it to ApplyUpdate
    if (tu && tu->IsUpdatable()) static_cast<UpdatableComponent *>(tu)->ApplyUpdate();
    h->sync();
    // the gradient is complete: to_update must not keep h's stream (h may be
    // destroyed before to_update's next DotProduct / Add waits on it)
    if (tu && tu->IsUpdatable()) static_cast<UpdatableComponent *>(tu)->ResetGradStream();
  });
}

long kctc_component_num_params(kctcComponent_t h) {
  return h && h->c->IsUpdatable() ? static_cast<UpdatableComponent &>(*h->c).NumParameters() : 0;
}

int kctc_component_get_params(kctcComponent_t h, float *host, long n) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h && host, "null argument");
    h->activate();
    auto &u = h->u();
    KCTC_REQUIRE(n == u.NumParameters(), "kctc_component_get_params: size mismatch");
    u.Vectorize(host);
  });
}

int kctc_component_set_params(kctcComponent_t h, const float *host, long n) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h && host, "null argument");
    h->activate();
    auto &u = h->u();
    KCTC_REQUIRE(n == u.NumParameters(), "kctc_component_set_params: size mismatch");
    u.UnVectorize(host);
    h->sync();
  });
}

int kctc_component_learning_rate(kctcComponent_t h, float *lr) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h && lr, "null argument");
    *lr = h->u().LearningRate();
  });
}

int kctc_component_set_learning_rate(kctcComponent_t h, float lr) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h, "null argument");
    h->u().SetLearningRate(lr);
  });
}

int kctc_component_is_gradient(kctcComponent_t h) {
  return h && h->c->IsUpdatable() && static_cast<UpdatableComponent &>(*h->c).IsGradient() ? 1 : 0;
}

int kctc_component_set_zero(kctcComponent_t h, int treat_as_gradient) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h, "null argument");
    h->activate();
    h->u().SetZero(treat_as_gradient != 0);
    h->sync();
  });
}

int kctc_component_dot_product(kctcComponent_t h, kctcComponent_t o, double *dot) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h && o && dot, "null argument");
    KCTC_REQUIRE(h->device == o->device, "kctc_component_dot_product: components on different devices");
    KCTC_HIP_CHECK(hipStreamSynchronize(o->stream));
    h->activate();
    *dot = h->u().DotProduct(o->u());
  });
}

int kctc_component_perturb_params(kctcComponent_t h, float stddev) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h, "null argument");
    h->activate();
    h->u().PerturbParams(stddev);
    h->sync();
  });
}

int kctc_component_scale(kctcComponent_t h, float scale) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h, "null argument");
    h->activate();
    scale_component(*h->c, scale);
    h->sync();
  });
}

int kctc_component_add(kctcComponent_t h, float alpha, kctcComponent_t o) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h && o, "null argument");
    KCTC_REQUIRE(h->device == o->device, "kctc_component_add: components on different devices");
    KCTC_HIP_CHECK(hipStreamSynchronize(o->stream));
    h->activate();
    add_component(*h->c, alpha, *o->c);
    h->sync();
  });
}

int kctc_set_perturb_seed(unsigned long long seed) {
  return kctc_guarded([&] { UpdatableComponent::SetPerturbSeed(seed); });
}

int kctc_component_srand(kctcComponent_t h, unsigned seed) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h, "null argument");
    h->rng.Seed(seed);
  });
}

int kctc_nnet_get_component(kctcNnet_t n, int index, kctcComponent_t *out) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(n && out, "null argument");
    KCTC_REQUIRE(index >= 0 && index < n->nnet.NumComponents(), "component index out of range");
    n->activate();
    KCTC_HIP_CHECK(hipStreamSynchronize(n->stream));
    if (n->side) KCTC_HIP_CHECK(hipStreamSynchronize(n->side));
    Component *c = n->nnet.GetComponent(index).Copy();
    KCTC_HIP_CHECK(hipStreamSynchronize(n->stream));
    *out = wrap(c, n->device);
  });
}

int kctc_nnet_set_component(kctcNnet_t n, int index, kctcComponent_t h) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(n && h, "null argument");
    KCTC_REQUIRE(n->trainer.Pending() == 0, "kctc_nnet_set_component with minibatches in flight");
    KCTC_REQUIRE(h->device == n->device, "kctc_nnet_set_component: component on another device");
    KCTC_HIP_CHECK(hipStreamSynchronize(h->stream));
    n->activate();
    KCTC_HIP_CHECK(hipStreamSynchronize(n->stream));
    if (n->side) KCTC_HIP_CHECK(hipStreamSynchronize(n->side));
    Component *c = h->c->Copy();
    if (n->nnet.Momentum() != 0.f) {
      if (c->IsUpdatable()) static_cast<UpdatableComponent *>(c)->SetMomentum(n->nnet.Momentum());
      if (auto *cg = dynamic_cast<ClipGradientComponent *>(c)) cg->EnableShadow(true);
    }
    n->nnet.SetComponent(index, c);
    KCTC_HIP_CHECK(hipStreamSynchronize(n->stream));
  });
}

int kctc_nnet_scale_params(kctcNnet_t n, float scale, int skip_last_layer) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(n, "null argument");
    KCTC_REQUIRE(n->trainer.Pending() == 0, "kctc_nnet_scale_params with minibatches in flight");
    n->activate();
    nnet_scale(n, scale, skip_last_layer != 0);
    KCTC_HIP_CHECK(hipStreamSynchronize(n->stream));
  });
}

int kctc_nnet_add_params(kctcNnet_t n, float alpha, kctcNnet_t other, int skip_last_layer) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(n && other, "null argument");
    KCTC_REQUIRE(n->device == other->device, "kctc_nnet_add_params: networks on different devices");
    KCTC_REQUIRE(n->trainer.Pending() == 0, "kctc_nnet_add_params with minibatches in flight");
    n->activate();
    nnet_add(n, alpha, other, skip_last_layer != 0);
    KCTC_HIP_CHECK(hipStreamSynchronize(n->stream));
  });
}

// nnet-am-average (nnet-am-average.cc:150-241): scale the first model's
// components by weights[0], then add weights[i] * model i in order
int kctc_nnet_average_models(kctcNnet_t *nnets, const float *weights, int num, int skip_last_layer) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(nnets && num >= 1, "kctc_nnet_average_models: no networks");
    for (int i = 0; i < num; i++) KCTC_REQUIRE(nnets[i], "kctc_nnet_average_models: null network");
    for (int i = 1; i < num; i++)
      KCTC_REQUIRE(nnets[i]->device == nnets[0]->device, "kctc_nnet_average_models: networks on different devices");
    std::vector<float> w(num, 1.0f / (float)num);  // GetWeights' default: 1/num-models
    if (weights) w.assign(weights, weights + num);
    // GetWeights (nnet-am-average.cc:45-53) normalises the weights to sum to one
    float wsum = 0.f;
    for (int i = 0; i < num; i++) wsum += w[i];
    KCTC_REQUIRE(wsum != 0.f && std::isfinite(wsum), "kctc_nnet_average_models: weights sum to zero");
    for (int i = 0; i < num; i++) w[i] /= wsum;
    kctcNnetImpl *avg = nnets[0];
    KCTC_REQUIRE(avg->trainer.Pending() == 0, "kctc_nnet_average_models with minibatches in flight");
    avg->activate();
    nnet_scale(avg, w[0], skip_last_layer != 0);
    for (int i = 1; i < num; i++) nnet_add(avg, w[i], nnets[i], skip_last_layer != 0);
    KCTC_HIP_CHECK(hipStreamSynchronize(avg->stream));
  });
}

// test hook (csrc/test_hooks.h): a CuDNNRecurrentComponent with the trainer's
// side streams and the forward-time prepacks of W^T (dx) and x^T / y^T (weights)
int kctc_test_component_side_streams(kctcComponent_t h, int on) {
  return kctc_guarded([&] {
    KCTC_REQUIRE(h, "kctc_test_component_side_streams: bad handle");
    auto *r = dynamic_cast<CuDNNRecurrentComponent *>(h->c.get());
    KCTC_REQUIRE(r, "kctc_test_component_side_streams: not a CuDNNRecurrentComponent");
    KCTC_HIP_CHECK(hipSetDevice(h->device));
    if (on && !h->side) {
      KCTC_HIP_CHECK(hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking));
      KCTC_HIP_CHECK(hipStreamCreateWithFlags(&h->stream2, hipStreamNonBlocking));
    }
    r->SetPrepackDx(on != 0);
    r->SetPrepackW(on != 0);
  });
}

}  // extern "C"
