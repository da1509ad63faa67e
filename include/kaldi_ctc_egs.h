/* kaldi_ctc_egs.h -- C ABI of the egs path: NnetCtcExample archives,
 * the CompressedMatrix codec, the background minibatch reader and
 * FormatNnetInput on the GPU (libkaldictc_amd.so, gfx950).
 *
 * Replaces (reference file:line):
 *   kctc_egs_writer_*        <- NnetCtcExampleWriter + NnetCtcExample::Write
 *                               (src/ctc/ctc-nnet-example.cc:29-44; used by
 *                               src/ctcbin/nnet-ctc-get-egs.cc), features kept as
 *                               CompressedMatrix (src/matrix/compressed-matrix.cc:41-123)
 *   kctc_egs_reader_*        <- SequentialNnetCtcExampleReader +
 *                               NnetCtcExampleBackgroundReader
 *                               (src/ctc/ctc-nnet-train.cc:31-183): a producer thread
 *                               reads the next minibatch while the caller trains;
 *                               skip rules num_frames > max_frames, labels > 639,
 *                               num_frames < 2*labels+1 (:84-95)
 *   kctc_minibatch_format    <- FormatNnetInput (src/ctc/ctc-nnet-update.cc:351-424)
 *                               + the H2D copy of ComputeForMinibatch (:94-128): the
 *                               compressed bytes are uploaded and decoded on the GPU
 *                               (CompressedMatrix::CopyToMat arithmetic, bit-exact)
 *   kctc_cm_compress/decompress <- CompressedMatrix::CopyFromMat / CopyToMat (host)
 *   kctc_egs_shuffle         <- nnet-ctc-shuffle-egs (src/ctcbin/nnet-ctc-shuffle-egs.cc:25-127)
 *                               + FrameSubsamplingShiftNnetCtcExampleTimes
 *                               (src/ctc/ctc-nnet-example.cc:78-106)
 *   kctc_egs_sort            <- nnet-ctc-sort-egs (src/ctcbin/nnet-ctc-sort-egs.cc:27-133)
 * Archives: binary Kaldi "ark" files ("ark:path" or a plain path).  Return 0 on
 * success, non-zero on error (kctc_last_error() in kaldi_ctc_train.h). */
#ifndef KALDI_CTC_EGS_H_
#define KALDI_CTC_EGS_H_

#ifdef __cplusplus
extern "C" {
#endif

typedef struct kctcEgsWriter_ *kctcEgsWriter_t;
typedef struct kctcEgsReader_ *kctcEgsReader_t;
typedef struct kctcMinibatch_ *kctcMinibatch_t;

/* --- CompressedMatrix codec (host) --- */
/* bytes of the in-memory image (GlobalHeader + body) of a rows x cols matrix */
long kctc_cm_compressed_bytes(int rows, int cols);
/* m: row-major rows x cols; out: kctc_cm_compressed_bytes(rows, cols) bytes */
int kctc_cm_compress(const float *m, int rows, int cols, void *out);
/* data: an image from kctc_cm_compress; out: rows x cols floats */
int kctc_cm_decompress(const void *data, float *out);

/* --- archive writer --- */
int kctc_egs_writer_open(kctcEgsWriter_t *w, const char *wspecifier);
/* one NnetCtcExample: feats row-major [num_rows][dim] (compressed on write),
 * labels[num_labels], left_context, spk_info[spk_dim] (spk_dim may be 0) */
int kctc_egs_write(kctcEgsWriter_t w, const char *key, const float *feats, int num_rows, int dim,
                   const int *labels, int num_labels, int left_context, const float *spk_info,
                   int spk_dim);
int kctc_egs_writer_close(kctcEgsWriter_t w);

/* --- egs preparation tools (host) --- */
/* Copy rspecifier -> wspecifier in the reference tools' order: --srand,
 * --buffer-size (0 = whole archive in memory), --frame-shift,
 * --frame-subsampling-factor (shuffle only; > 1 keeps input rows
 * frame_shift, frame_shift + f, ... and re-compresses).  *num_done = examples
 * written (the tools exit with status 1 when it is 0). */
int kctc_egs_shuffle(const char *rspecifier, const char *wspecifier, int srand_seed, int buffer_size,
                     int frame_shift, int frame_subsampling_factor, long *num_done);
int kctc_egs_sort(const char *rspecifier, const char *wspecifier, int srand_seed, int buffer_size,
                  long *num_done);

/* --- background minibatch reader --- */
/* nnet_left_context / nnet_right_context: the network's context (0 for the
 * recipe's splice-0 input; FormatNnetInput's num_splice = 1 + both) */
int kctc_egs_reader_open(kctcEgsReader_t *r, const char *rspecifier, int minibatch_size,
                         int max_frames, int nnet_left_context, int nnet_right_context);
/* next minibatch; *mb = NULL when the archive is exhausted.  The caller owns
 * *mb (kctc_minibatch_free). */
int kctc_egs_reader_next(kctcEgsReader_t r, kctcMinibatch_t *mb);
int kctc_egs_reader_stats(kctcEgsReader_t r, long *num_read, long *num_skipped);
int kctc_egs_reader_close(kctcEgsReader_t r);

/* --- a minibatch --- */
int kctc_minibatch_info(kctcMinibatch_t mb, int *N, int *T_max, int *input_dim, long *total_labels);
/* rows per output frame of the formatted input: 1 + the nnet left + right
 * context the reader was opened with (FormatNnetInput's num_splice) */
int kctc_minibatch_num_splice(kctcMinibatch_t mb);
/* num_frames[N], label_lengths[N], flat_labels[total_labels] (host) */
int kctc_minibatch_labels(kctcMinibatch_t mb, int *num_frames, int *label_lengths, int *flat_labels);
/* key of example n (pointer valid until kctc_minibatch_free) */
const char *kctc_minibatch_key(kctcMinibatch_t mb, int n);
long kctc_minibatch_scratch_bytes(kctcMinibatch_t mb);
/* stream-ordered: upload the compressed bytes into scratch (device) and decode
 * into out (device) [T_max*N][input_dim], row t*N+n, zero for t >= T_n.  The
 * minibatch must outlive the copy (kctc_minibatch_free waits for it). */
int kctc_minibatch_format(kctcMinibatch_t mb, float *out, void *scratch, long scratch_bytes,
                          void *stream);
int kctc_minibatch_free(kctcMinibatch_t mb);

#ifdef __cplusplus
}
#endif

#endif /* KALDI_CTC_EGS_H_ */
