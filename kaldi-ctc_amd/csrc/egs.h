// egs.h -- NnetCtcExample archives, the CompressedMatrix codec and the
// background minibatch reader (host side of the egs path).
//
//   NnetCtcExample::Write/Read        src/ctc/ctc-nnet-example.cc:29-60
//   CompressedMatrix (format 1 / 2)   src/matrix/compressed-matrix.{h:128-171, cc:27-540}
//   NnetCtcExampleBackgroundReader    src/ctc/ctc-nnet-train.cc:31-183
//   FormatNnetInput                   src/ctc/ctc-nnet-update.cc:351-424 (decode + pack
//                                     run on the GPU: egs_format.hip)
//
// The compressed bytes are kept as they are on disk; the reader only parses
// headers, applies the reference's skip rules and packs a minibatch into one
// contiguous host blob, which the GPU decodes straight into the time-major
// [T_max*N][dim] network input.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <fstream>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace kctc {
namespace egs {

// CompressedMatrix::GlobalHeader (compressed-matrix.h:128-134); format 1 =
// per-column percentile headers + one byte per element (column-major),
// format 2 (<= 8 rows) = uint16 per element (row-major).
struct CmHeader {
  int32_t format;
  float min_value;
  float range;
  int32_t num_rows;
  int32_t num_cols;
};
static_assert(sizeof(CmHeader) == 20, "GlobalHeader is 20 bytes");

struct CmPerCol {
  uint16_t p0, p25, p75, p100;
};

// bytes of the data that follow the GlobalHeader
size_t cm_body_bytes(const CmHeader &h);
// CompressedMatrix::CopyFromMat (compressed-matrix.cc:41-123): header + body
std::vector<uint8_t> cm_compress(const float *m, int rows, int cols);
// CompressedMatrix::CopyToMat (host; the device decoder is egs_format.hip)
void cm_decompress(const uint8_t *data, float *out);

// One parsed example.  `cm` holds GlobalHeader + body (the compressed matrix
// as the reference keeps it in memory).
struct Example {
  std::string key;
  std::vector<int32_t> labels;
  std::vector<uint8_t> cm;
  int32_t left_context = 0;
  std::vector<float> spk_info;
  int NumFrames() const;
  int NumCols() const;
};

// Kaldi binary archive I/O ("ark:" or a plain path; binary mode only, which is
// what nnet-ctc-get-egs writes).
class ArchiveReader {
 public:
  explicit ArchiveReader(const std::string &rspecifier);
  bool Next(Example *eg);  // false at end of archive
 private:
  std::ifstream is_;
  std::string path_;
};

class ArchiveWriter {
 public:
  explicit ArchiveWriter(const std::string &wspecifier);
  void Write(const Example &eg);
  void Close();
 private:
  std::ofstream os_;
};

// Per-example descriptor for the device decoder.
struct EgDesc {
  int64_t off;      // byte offset of the body in the blob (16-B aligned)
  int32_t format;   // 1 or 2
  int32_t rows;     // CompressedMatrix rows
  int32_t cols;     // feature dim
  float min_value, range;
  int32_t first;    // first row used (ignore_frames)
  int32_t frames;   // frames copied (T_n)
  int64_t spk_off;  // byte offset of spk_info floats in the blob (-1: none)
  int32_t pad[2];
};
static_assert(sizeof(EgDesc) == 56, "EgDesc layout");

// A formatted-on-demand minibatch: everything FormatNnetInput needs, still
// compressed.  The blob is [EgDesc x N][bodies...] so one H2D copy moves it.
struct Minibatch {
  std::vector<std::string> keys;
  std::vector<int32_t> num_frames, label_lengths, labels;
  int N = 0, T_max = 0, feat_dim = 0, spk_dim = 0;
  int num_splice = 1;  // 1 + nnet left + right context: rows per output frame of the formatted input
  std::vector<uint8_t> blob;
  hipEvent_t done = nullptr;  // recorded after the last use of `blob` by a copy
  ~Minibatch();
  int InputDim() const { return feat_dim + spk_dim; }
};

// FormatNnetInput bookkeeping for a vector of examples (num_splice = 1 +
// nnet left/right context, ignore_frames = left_context - nnet_left_context).
std::unique_ptr<Minibatch> pack_minibatch(std::vector<Example> &egs, int nnet_left_context,
                                          int nnet_right_context);

// NnetCtcExampleBackgroundReader: a producer thread reads and packs the next
// minibatch while the caller trains on the current one (one slot, two
// semaphores' worth of hand-off).  Skip rules of ctc-nnet-train.cc:84-95.
class BackgroundReader {
 public:
  BackgroundReader(const std::string &rspecifier, int minibatch_size, int max_frames,
                   int nnet_left_context, int nnet_right_context);
  ~BackgroundReader();
  // nullptr when the archive is exhausted
  std::unique_ptr<Minibatch> Next();
  long NumSkipped() const { return skipped_; }
  long NumRead() const { return read_; }

 private:
  void Run();
  ArchiveReader reader_;
  int minibatch_size_, max_frames_, left_, right_;
  std::thread thread_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::unique_ptr<Minibatch> slot_;
  bool slot_full_ = false, finished_ = false, stop_ = false;
  std::string error_;
  long skipped_ = 0, read_ = 0;
};

// Egs preparation tools (egs_tools.cpp): nnet-ctc-shuffle-egs
// (src/ctcbin/nnet-ctc-shuffle-egs.cc:25-127) and nnet-ctc-sort-egs
// (src/ctcbin/nnet-ctc-sort-egs.cc:27-133), same example order as the reference
// binaries (glibc rand stream, libstdc++ shuffle / sort).  Return the number of
// examples written.
void FrameSubsamplingShift(int frame_subsampling_factor, int frame_shift, Example *eg);
long ShuffleEgs(const std::string &rspecifier, const std::string &wspecifier, int srand_seed,
                int buffer_size, int frame_shift, int frame_subsampling_factor);
long SortEgs(const std::string &rspecifier, const std::string &wspecifier, int srand_seed,
             int buffer_size);

// Device side (egs_format.hip).
size_t format_scratch_bytes(const Minibatch &mb);
// H2D copy of the blob into `scratch`, then decode + pack into out[T_max*N][dim]
// (row t*N+n, zero for t >= T_n), stream-ordered.
void format_on_device(Minibatch &mb, float *out, void *scratch, size_t scratch_bytes,
                      hipStream_t stream);

}  // namespace egs
}  // namespace kctc

// opaque handles of include/kaldi_ctc_egs.h (shared by egs_api.cpp and train_api.cpp)
struct kctcEgsReader_ {
  kctc::egs::BackgroundReader r;
  kctcEgsReader_(const char *spec, int mb, int max_frames, int l, int rc) : r(spec, mb, max_frames, l, rc) {}
};
