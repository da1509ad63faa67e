// rnn_api.cpp -- C ABI of include/kaldi_rnn.h over the gfx950 RNN layer (rnn.hip).
#include "kaldi_rnn.h"

#include <hip/hip_runtime.h>

#include <exception>
#include <new>

#include "common.h"
#include "rnn.h"

struct krnnContext {
  kctc::RnnDesc desc;
  unsigned *err = nullptr;  // device error word of the persistent kernels
  unsigned *dev_err() {
    if (!err) {
      KCTC_HIP_CHECK(hipMalloc(&err, 256));
      KCTC_HIP_CHECK(hipMemset(err, 0, 256));
    }
    return err;
  }
};


extern "C" {

int krnnCreate(krnnDescriptor_t *desc, int mode, int input_dim, int hidden_dim, int num_layers,
               int bidirectional) {
  if (!desc || mode < 0 || mode > 3 || input_dim <= 0 || hidden_dim <= 0 || num_layers <= 0)
    return KRNN_STATUS_BAD_PARAM;
  krnnContext *c = new (std::nothrow) krnnContext;
  if (!c) return KRNN_STATUS_EXECUTION_FAILED;
  c->desc.mode = mode;
  c->desc.D = input_dim;
  c->desc.H = hidden_dim;
  c->desc.layers = num_layers;
  c->desc.dirs = bidirectional ? 2 : 1;
  *desc = c;  // the device error word is allocated on first use (no GPU needed here)
  return KRNN_STATUS_SUCCESS;
}

int krnnSetPrecision(krnnDescriptor_t desc, int precision) {
  if (!desc || (precision != KRNN_PREC_FP32 && precision != KRNN_PREC_BF16)) return KRNN_STATUS_BAD_PARAM;
  if (precision == KRNN_PREC_BF16 && desc->desc.mode != kctc::kLstm && desc->desc.mode != kctc::kGru)
    return KRNN_STATUS_NOT_SUPPORTED;
  kctc::rnn_set_precision(desc->desc, precision);
  return KRNN_STATUS_SUCCESS;
}

int krnnDestroy(krnnDescriptor_t desc) {
  if (!desc) return KRNN_STATUS_BAD_PARAM;
  if (desc->err) (void)hipFree(desc->err);
  delete desc;
  return KRNN_STATUS_SUCCESS;
}

const char *krnnGetStatusString(int status) {
  switch (status) {
    case KRNN_STATUS_SUCCESS: return "success";
    case KRNN_STATUS_BAD_PARAM: return "bad parameter";
    case KRNN_STATUS_NOT_SUPPORTED: return "configuration not supported";
    case KRNN_STATUS_EXECUTION_FAILED: return "execution failed";
    case KRNN_STATUS_TIMEOUT: return "recurrence hand-off timed out";
    default: return "unknown status";
  }
}

size_t krnnGetParamsSize(krnnDescriptor_t desc) {
  return desc ? sizeof(float) * (size_t)desc->desc.params_size() : 0;
}

long krnnGetLinLayerOffset(krnnDescriptor_t desc, int pseudo_layer, int lin_layer_id, int is_bias,
                           int *dims) {
  if (!desc) return -1;
  const kctc::RnnDesc &d = desc->desc;
  const int nlin = 2 * d.nw();
  if (pseudo_layer < 0 || pseudo_layer >= d.layers * d.dirs || lin_layer_id < 0 ||
      lin_layer_id >= nlin)
    return -1;
  if (dims) {
    dims[0] = d.H;
    dims[1] = is_bias ? 1 : (lin_layer_id < d.nw() ? d.din(pseudo_layer / d.dirs) : d.H);
  }
  return d.lin_offset(pseudo_layer, lin_layer_id, is_bias != 0);
}

size_t krnnGetTrainingReserveSize(krnnDescriptor_t desc, int seq_length, int minibatch) {
  if (!desc || seq_length <= 0 || minibatch <= 0) return 0;
  return sizeof(float) * (size_t)kctc::rnn_reserve_layout(desc->desc, seq_length, minibatch).total;
}

size_t krnnGetWorkspaceSize(krnnDescriptor_t desc, int seq_length, int minibatch) {
  // scratch of the weight-gradient GEMMs; plus room for the per-step gate
  // activations that ForwardInference keeps (it has no reserve argument).
  if (!desc || seq_length <= 0 || minibatch <= 0) return 0;
  return kctc::rnn_workspace_bytes(desc->desc, seq_length, minibatch) +
         krnnGetTrainingReserveSize(desc, seq_length, minibatch);
}

int krnnForwardTraining(krnnDescriptor_t desc, struct ihipStream_t *stream, int seq_length,
                        int minibatch, const float *x, const float *w, float *y, void *workspace,
                        size_t workspace_bytes, void *reserve, size_t reserve_bytes) {
  if (!desc || !x || !w || !y || !reserve) return KRNN_STATUS_BAD_PARAM;
  try {
    return kctc::rnn_forward_training(desc->desc, stream, seq_length, minibatch, x, w, y, workspace,
                                      workspace_bytes, reserve, reserve_bytes, desc->dev_err());
  } catch (...) {
    return KRNN_STATUS_EXECUTION_FAILED;
  }
}

int krnnForwardInference(krnnDescriptor_t desc, struct ihipStream_t *stream, int seq_length,
                         int minibatch, const float *x, const float *w, float *y, void *workspace,
                         size_t workspace_bytes) {
  if (!desc || !x || !w || !y || !workspace) return KRNN_STATUS_BAD_PARAM;
  const size_t scratch = kctc::rnn_workspace_bytes(desc->desc, seq_length, minibatch);
  if (workspace_bytes < krnnGetWorkspaceSize(desc, seq_length, minibatch))
    return KRNN_STATUS_BAD_PARAM;
  char *ws = static_cast<char *>(workspace);
  try {
    return kctc::rnn_forward_training(desc->desc, stream, seq_length, minibatch, x, w, y, ws,
                                      scratch, ws + kctc::align_up(scratch, 256),
                                      workspace_bytes - kctc::align_up(scratch, 256), desc->dev_err());
  } catch (...) {
    return KRNN_STATUS_EXECUTION_FAILED;
  }
}

int krnnBackwardData(krnnDescriptor_t desc, struct ihipStream_t *stream, int seq_length,
                     int minibatch, const float *y, const float *dy, const float *w, float *dx,
                     void *workspace, size_t workspace_bytes, void *reserve,
                     size_t reserve_bytes) {
  if (!desc || !y || !dy || !w || !reserve) return KRNN_STATUS_BAD_PARAM;
  try {
    return kctc::rnn_backward_data(desc->desc, stream, seq_length, minibatch, y, dy, w, dx,
                                   workspace, workspace_bytes, reserve, reserve_bytes, desc->dev_err());
  } catch (...) {
    return KRNN_STATUS_EXECUTION_FAILED;
  }
}

int krnnBackwardWeights(krnnDescriptor_t desc, struct ihipStream_t *stream, int seq_length,
                        int minibatch, const float *x, const float *y, void *workspace,
                        size_t workspace_bytes, float *dw, void *reserve, size_t reserve_bytes) {
  if (!desc || !x || !y || !dw || !reserve || !workspace) return KRNN_STATUS_BAD_PARAM;
  try {
    return kctc::rnn_backward_weights(desc->desc, stream, seq_length, minibatch, x, y, workspace,
                                      workspace_bytes, dw, reserve, reserve_bytes);
  } catch (...) {
    return KRNN_STATUS_EXECUTION_FAILED;
  }
}

int krnnGetDeviceStatus(krnnDescriptor_t desc, struct ihipStream_t *stream) {
  if (!desc) return KRNN_STATUS_BAD_PARAM;
  unsigned e = 0;
  if (!desc->err) return KRNN_STATUS_SUCCESS;
  if (hipMemcpyAsync(&e, desc->err, sizeof(e), hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess)
    return KRNN_STATUS_EXECUTION_FAILED;
  if (e) {
    (void)hipMemsetAsync(desc->err, 0, sizeof(unsigned), stream);
    return KRNN_STATUS_TIMEOUT;
  }
  return KRNN_STATUS_SUCCESS;
}

}  // extern "C"
