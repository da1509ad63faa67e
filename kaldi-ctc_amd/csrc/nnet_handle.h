// nnet_handle.h -- the object behind the kctcNnet_t handle of
// include/kaldi_ctc_train.h (shared by train_api.cpp and component_api.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "common.h"
#include "kaldi_ctc_train.h"
#include "nnet.h"

struct kctcNnetImpl {
  int device = 0;
  hipStream_t stream = nullptr;
  kctc::nnet2::Nnet nnet;
  kctc::nnet2::NnetCtcUpdater trainer{&nnet, true};
  kctc::nnet2::NnetCtcUpdater evaluator{&nnet, false};
  hipStream_t side = nullptr, stream2 = nullptr;
  kctc::nnet2::GradExchange *dp = nullptr;
  bool dp_average = false;  // model averaging: no per-step gradient exchange
  kctc::nnet2::DevBuf egs_feats, egs_scratch;  // TrainNnetSimple staging
  // decodable (per utterance): device priors, uploaded again only when they
  // change, and the output / scratch buffers, grown and kept
  kctc::nnet2::DevBuf dec_priors, dec_out, dec_scratch, dec_input;
  std::vector<float> dec_priors_host;
  // nnet2-ctc model file extras: the CtcTransitionModel exactly as read (opaque
  // bytes, in the mode of the file it came from) and AmNnet's priors
  std::string trans_model;
  bool trans_model_binary = false;
  std::vector<float> priors;
  ~kctcNnetImpl() {
    delete dp;
    if (stream) (void)hipStreamSynchronize(stream);
    if (side) (void)hipStreamSynchronize(side);
    if (stream2) (void)hipStreamSynchronize(stream2);
    auto &d = kctc::nnet2::CuDevice::Instantiate();
    if (d.stream == stream) d.stream = nullptr;
    if (d.side == side) d.side = nullptr;
    if (d.stream2 == stream2) d.stream2 = nullptr;
    if (stream) (void)hipStreamDestroy(stream);
    if (side) (void)hipStreamDestroy(side);
    if (stream2) (void)hipStreamDestroy(stream2);
  }
  // compute stream at the highest priority (the latency-bound recurrences),
  // the weight-gradient side stream at the lowest (train_api.cpp)
  void create_streams();
  void activate() {
    KCTC_HIP_CHECK(hipSetDevice(device));
    auto &d = kctc::nnet2::CuDevice::Instantiate();
    d.device = device;
    d.stream = stream;
    d.side = side;
    d.stream2 = stream2;
  }
};

// kctc_last_error() text of the calling thread (train_api.cpp)
void kctc_set_error(const char *msg);

// runs f, mapping exceptions to a non-zero return and kctc_last_error()
template <typename F>
int kctc_guarded(F f) {
  try {
    f();
    return 0;
  } catch (const std::exception &e) {
    kctc_set_error(e.what());
    return 1;
  } catch (...) {
    kctc_set_error("unknown error");
    return 1;
  }
}
