/*
 * kaldi_rnn.h -- cuDNN-shaped C ABI for the recurrent layer, implemented by
 * libkaldictc_amd.so with hand-written gfx950 HIP kernels (rnn.hip, gemm.hip).
 *
 * Replaces the kaldi::cudnn shim over cuDNN 5.1 used by CuDNNRecurrentComponent:
 *   krnnGetParamsSize           <- cudnn::GetRecurrentParamsSize
 *                                  (src/cudamatrix/cudnn-recurrent.h:113-117, called
 *                                   at src/nnet2/nnet-cudnn-component.cc:270-273)
 *   krnnGetLinLayerOffset       <- cudnn::GetRecurrentLinLayerMatrixParams /
 *                                  GetRecurrentLinLayerBiasParams (cudnn-recurrent.h:119-139,
 *                                  nnet-cudnn-component.cc:336-407, 417-483)
 *   krnnGetWorkspaceSize        <- cudnn::GetRecurrentWorkspaceSize (cudnn-recurrent.h:101-105)
 *   krnnGetTrainingReserveSize  <- cudnn::GetRecurrentTrainingReserveSize (:107-111)
 *   krnnForwardTraining         <- cudnn::RecurrentForwardTraining (:34-53,
 *                                  nnet-cudnn-component.cc:545-554)
 *   krnnForwardInference        <- cudnn::RecurrentForwardInference (:15-32, :534-543)
 *   krnnBackwardData            <- cudnn::RecurrentBackwardData (:55-80, :576-588)
 *   krnnBackwardWeights         <- cudnn::RecurrentBackwardWeights (:83-97, :594-599)
 *
 * Conventions (identical to the reference's use of cuDNN):
 *   x [T][N][input_dim], y [T][N][dirs*hidden] (forward direction in columns
 *   0..H-1), fp32, contiguous, time-major -- the FormatNnetInput layout.  All N
 *   sequences run T steps (no masking).  Initial/final states: the reference
 *   zeroes hx/cx/dhy/dcy before every call and never reads hy/cy/dhx/dcx
 *   (nnet-cudnn-component.cc:494-506), so this ABI has no state arguments:
 *   hx = cx = dhy = dcy = 0.  Weights use the cuDNN v5 opaque layout: per
 *   pseudo-layer (layer*dirs + dir) the nlin matrices (input W [H][Din] for
 *   ids < nlin/2, recurrent R [H][H] above; LSTM ids i,f,c,o / GRU r,z,h) then
 *   the nlin bias vectors [H].  BackwardWeights ACCUMULATES into dw.
 *   BackwardData must follow ForwardTraining with the same reserve, and
 *   BackwardWeights must follow BackwardData (it consumes the gate gradients
 *   BackwardData leaves in the reserve), as with cuDNN.
 *   Every call is ordered on `stream`; none synchronises the host.  Return 0 on
 *   success, a KRNN_STATUS_* code otherwise.
 */
#ifndef KALDI_CTC_AMD_KALDI_RNN_H_
#define KALDI_CTC_AMD_KALDI_RNN_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

struct ihipStream_t;

typedef enum { KRNN_RELU = 0, KRNN_TANH = 1, KRNN_LSTM = 2, KRNN_GRU = 3 } krnnMode_t;

typedef enum {
  KRNN_STATUS_SUCCESS = 0,
  KRNN_STATUS_BAD_PARAM = 1,
  KRNN_STATUS_NOT_SUPPORTED = 2,
  KRNN_STATUS_EXECUTION_FAILED = 3,
  KRNN_STATUS_TIMEOUT = 4
} krnnStatus_t;

typedef struct krnnContext *krnnDescriptor_t;

int krnnCreate(krnnDescriptor_t *desc, int mode, int input_dim, int hidden_dim, int num_layers,
               int bidirectional);
int krnnDestroy(krnnDescriptor_t desc);
/* Arithmetic of the recurrences and gate GEMMs (an extension; cuDNN 5 has
 * no such switch): KRNN_PREC_FP32 (default) -- fp32-class products (split-fp16
 * pairs, fp32 accumulation); KRNN_PREC_BF16 -- bf16 operands, fp32
 * accumulation and master weights (LSTM / GRU only, BASELINE configs[4]). */
enum { KRNN_PREC_FP32 = 0, KRNN_PREC_BF16 = 1 };
int krnnSetPrecision(krnnDescriptor_t desc, int precision);
/* (as cuDNN's data type, precision is part of the descriptor: query the
 * workspace / reserve sizes after setting it -- a one-layer bf16 reserve also
 * holds the recurrences' packed GEMM operands, KCTC_BF16_DIRECT=0 drops them) */
const char *krnnGetStatusString(int status);

/* bytes of the opaque weight buffer (cudnnGetRNNParamsSize) */
size_t krnnGetParamsSize(krnnDescriptor_t desc);
/* float offset of lin layer `lin_layer_id` of pseudo-layer `pseudo_layer` in the
 * weight buffer; dims[0..1] = rows, cols ([H][Din], [H][H] or [H][1] for a bias). */
long krnnGetLinLayerOffset(krnnDescriptor_t desc, int pseudo_layer, int lin_layer_id,
                           int is_bias, int *dims);
size_t krnnGetWorkspaceSize(krnnDescriptor_t desc, int seq_length, int minibatch);
size_t krnnGetTrainingReserveSize(krnnDescriptor_t desc, int seq_length, int minibatch);

int krnnForwardTraining(krnnDescriptor_t desc, struct ihipStream_t *stream, int seq_length,
                        int minibatch, const float *x, const float *w, float *y,
                        void *workspace, size_t workspace_bytes, void *reserve,
                        size_t reserve_bytes);
int krnnForwardInference(krnnDescriptor_t desc, struct ihipStream_t *stream, int seq_length,
                         int minibatch, const float *x, const float *w, float *y,
                         void *workspace, size_t workspace_bytes);
int krnnBackwardData(krnnDescriptor_t desc, struct ihipStream_t *stream, int seq_length,
                     int minibatch, const float *y, const float *dy, const float *w, float *dx,
                     void *workspace, size_t workspace_bytes, void *reserve,
                     size_t reserve_bytes);
int krnnBackwardWeights(krnnDescriptor_t desc, struct ihipStream_t *stream, int seq_length,
                        int minibatch, const float *x, const float *y, void *workspace,
                        size_t workspace_bytes, float *dw, void *reserve, size_t reserve_bytes);
/* Reads (and clears) the device error word of the persistent recurrence
 * kernels: KRNN_STATUS_TIMEOUT if a bounded spin gave up.  Synchronises. */
int krnnGetDeviceStatus(krnnDescriptor_t desc, struct ihipStream_t *stream);

#ifdef __cplusplus
}
#endif
#endif /* KALDI_CTC_AMD_KALDI_RNN_H_ */
