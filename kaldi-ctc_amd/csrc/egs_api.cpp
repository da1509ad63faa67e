// egs_api.cpp -- C ABI of include/kaldi_ctc_egs.h.
#include "kaldi_ctc_egs.h"

#include <cstring>
#include <string>

#include "common.h"
#include "egs.h"

using namespace kctc::egs;

struct kctcEgsWriter_ {
  ArchiveWriter w;
  explicit kctcEgsWriter_(const char *spec) : w(spec) {}
};
struct kctcMinibatch_ {
  std::unique_ptr<Minibatch> mb;
};

// shared with train_api.cpp (kctc_last_error)
void kctc_set_error(const char *msg);

template <typename F>
static int guarded(F f) {
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

extern "C" {

long kctc_cm_compressed_bytes(int rows, int cols) {
  if (rows <= 0 || cols <= 0) return 0;
  CmHeader h{};
  h.format = rows > 8 ? 1 : 2;
  h.num_rows = rows;
  h.num_cols = cols;
  return (long)(sizeof(CmHeader) + cm_body_bytes(h));
}

int kctc_cm_compress(const float *m, int rows, int cols, void *out) {
  return guarded([&] {
    KCTC_REQUIRE(m && out && rows > 0 && cols > 0, "kctc_cm_compress: bad arguments");
    auto v = cm_compress(m, rows, cols);
    memcpy(out, v.data(), v.size());
  });
}

int kctc_cm_decompress(const void *data, float *out) {
  return guarded([&] {
    KCTC_REQUIRE(data && out, "kctc_cm_decompress: bad arguments");
    cm_decompress(static_cast<const uint8_t *>(data), out);
  });
}

int kctc_egs_writer_open(kctcEgsWriter_t *w, const char *spec) {
  return guarded([&] {
    KCTC_REQUIRE(w && spec, "kctc_egs_writer_open: bad arguments");
    *w = new kctcEgsWriter_(spec);
  });
}

int kctc_egs_write(kctcEgsWriter_t w, const char *key, const float *feats, int num_rows, int dim,
                   const int *labels, int num_labels, int left_context, const float *spk_info, int spk_dim) {
  return guarded([&] {
    KCTC_REQUIRE(w && key && num_rows >= 0 && dim >= 0 && num_labels >= 0 && spk_dim >= 0,
                 "kctc_egs_write: bad arguments");
    Example eg;
    eg.key = key;
    eg.labels.assign(labels, labels + num_labels);
    if (num_rows > 0 && dim > 0) eg.cm = cm_compress(feats, num_rows, dim);
    eg.left_context = left_context;
    if (spk_dim) eg.spk_info.assign(spk_info, spk_info + spk_dim);
    w->w.Write(eg);
  });
}

int kctc_egs_writer_close(kctcEgsWriter_t w) {
  return guarded([&] {
    if (!w) return;
    w->w.Close();
    delete w;
  });
}

int kctc_egs_shuffle(const char *rspecifier, const char *wspecifier, int srand_seed, int buffer_size,
                     int frame_shift, int frame_subsampling_factor, long *num_done) {
  return guarded([&] {
    KCTC_REQUIRE(rspecifier && wspecifier, "kctc_egs_shuffle: null specifier");
    const long n = ShuffleEgs(rspecifier, wspecifier, srand_seed, buffer_size, frame_shift,
                              frame_subsampling_factor);
    if (num_done) *num_done = n;
  });
}

int kctc_egs_sort(const char *rspecifier, const char *wspecifier, int srand_seed, int buffer_size,
                  long *num_done) {
  return guarded([&] {
    KCTC_REQUIRE(rspecifier && wspecifier, "kctc_egs_sort: null specifier");
    const long n = SortEgs(rspecifier, wspecifier, srand_seed, buffer_size);
    if (num_done) *num_done = n;
  });
}

int kctc_egs_reader_open(kctcEgsReader_t *r, const char *spec, int minibatch_size, int max_frames, int l,
                         int rc) {
  return guarded([&] {
    KCTC_REQUIRE(r && spec, "kctc_egs_reader_open: bad arguments");
    *r = new kctcEgsReader_(spec, minibatch_size, max_frames, l, rc);
  });
}

int kctc_egs_reader_next(kctcEgsReader_t r, kctcMinibatch_t *mb) {
  return guarded([&] {
    KCTC_REQUIRE(r && mb, "kctc_egs_reader_next: bad arguments");
    *mb = nullptr;
    auto m = r->r.Next();
    if (m) {
      *mb = new kctcMinibatch_;
      (*mb)->mb = std::move(m);
    }
  });
}

int kctc_egs_reader_stats(kctcEgsReader_t r, long *num_read, long *num_skipped) {
  return guarded([&] {
    KCTC_REQUIRE(r, "kctc_egs_reader_stats: bad arguments");
    if (num_read) *num_read = r->r.NumRead();
    if (num_skipped) *num_skipped = r->r.NumSkipped();
  });
}

int kctc_egs_reader_close(kctcEgsReader_t r) {
  return guarded([&] { delete r; });
}

int kctc_minibatch_info(kctcMinibatch_t m, int *N, int *T_max, int *input_dim, long *total_labels) {
  return guarded([&] {
    KCTC_REQUIRE(m && m->mb, "kctc_minibatch_info: bad minibatch");
    const Minibatch &b = *m->mb;
    if (N) *N = b.N;
    if (T_max) *T_max = b.T_max;
    if (input_dim) *input_dim = b.InputDim();
    if (total_labels) *total_labels = (long)b.labels.size();
  });
}

int kctc_minibatch_num_splice(kctcMinibatch_t m) { return m && m->mb ? m->mb->num_splice : -1; }

int kctc_minibatch_labels(kctcMinibatch_t m, int *num_frames, int *label_lengths, int *flat_labels) {
  return guarded([&] {
    KCTC_REQUIRE(m && m->mb, "kctc_minibatch_labels: bad minibatch");
    const Minibatch &b = *m->mb;
    if (num_frames) memcpy(num_frames, b.num_frames.data(), sizeof(int) * b.N);
    if (label_lengths) memcpy(label_lengths, b.label_lengths.data(), sizeof(int) * b.N);
    if (flat_labels && !b.labels.empty()) memcpy(flat_labels, b.labels.data(), sizeof(int) * b.labels.size());
  });
}

const char *kctc_minibatch_key(kctcMinibatch_t m, int n) {
  if (!m || !m->mb || n < 0 || n >= m->mb->N) return nullptr;
  return m->mb->keys[n].c_str();
}

long kctc_minibatch_scratch_bytes(kctcMinibatch_t m) {
  if (!m || !m->mb) return -1;
  return (long)format_scratch_bytes(*m->mb);
}

int kctc_minibatch_format(kctcMinibatch_t m, float *out, void *scratch, long scratch_bytes, void *stream) {
  return guarded([&] {
    KCTC_REQUIRE(m && m->mb && out && scratch && scratch_bytes >= 0, "kctc_minibatch_format: bad arguments");
    format_on_device(*m->mb, out, scratch, (size_t)scratch_bytes, static_cast<hipStream_t>(stream));
  });
}

int kctc_minibatch_free(kctcMinibatch_t m) {
  return guarded([&] { delete m; });
}

}  // extern "C"
