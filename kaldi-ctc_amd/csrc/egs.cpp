// egs.cpp -- NnetCtcExample archives, CompressedMatrix encoder and the
// background minibatch reader (see egs.h for the reference map).
#include "egs.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "common.h"

// The codec's rounding is part of the on-disk format: keep every product and
// sum a separately rounded operation, as the reference's x86 build does.
#pragma clang fp contract(off)

namespace kctc {
namespace egs {

// ---------------------------------------------------------------------------
// CompressedMatrix codec (compressed-matrix.cc:27-38, 41-123, 193-335)
// ---------------------------------------------------------------------------
size_t cm_body_bytes(const CmHeader &h) {
  if (h.format == 1) return (size_t)h.num_cols * (sizeof(CmPerCol) + (size_t)h.num_rows);
  if (h.format == 2) return 2 * (size_t)h.num_rows * h.num_cols;
  throw std::runtime_error("CompressedMatrix: bad format " + std::to_string(h.format));
}

static inline uint16_t to_u16(const CmHeader &h, float v) {
  float f = (v - h.min_value) / h.range;
  if (f > 1.0f) f = 1.0f;
  if (f < 0.0f) f = 0.0f;
  return (uint16_t)(int)((double)(f * 65535.0f) + 0.499);
}

static inline float from_u16(const CmHeader &h, uint16_t v) {
  const float a = h.range * 1.52590218966964e-05F;
  return h.min_value + a * (float)v;
}

static inline uint8_t to_u8(float p0, float p25, float p75, float p100, float v) {
  int ans;
  if (v < p25) {
    const float f = (v - p0) / (p25 - p0);
    ans = (int)((double)(f * 64.0f) + 0.5);
    ans = std::min(64, std::max(0, ans));
  } else if (v < p75) {
    const float f = (v - p25) / (p75 - p25);
    ans = 64 + (int)((double)(f * 128.0f) + 0.5);
    ans = std::min(192, std::max(64, ans));
  } else {
    const float f = (v - p75) / (p100 - p75);
    ans = 192 + (int)((double)(f * 63.0f) + 0.5);
    ans = std::min(255, std::max(192, ans));
  }
  return (uint8_t)ans;
}

static inline float from_u8(float p0, float p25, float p75, float p100, uint8_t v) {
  if (v <= 64) return (float)((double)p0 + (double)((p25 - p0) * (float)v) * (1 / 64.0));
  if (v <= 192) return (float)((double)p25 + (double)((p75 - p25) * (float)(v - 64)) * (1 / 128.0));
  return (float)((double)p75 + (double)((p100 - p75) * (float)(v - 192)) * (1 / 63.0));
}

// percentiles of one column: order statistics 0, n/4, 3n/4, n-1 (the
// reference gets them with nth_element; any selection gives the same values)
static CmPerCol col_header(const CmHeader &h, std::vector<float> &col) {
  const int n = (int)col.size();
  CmPerCol c;
  std::sort(col.begin(), col.end());
  if (n >= 5) {
    const int q = n / 4;
    c.p0 = std::min<uint16_t>(to_u16(h, col[0]), 65532);
    c.p25 = std::min<uint16_t>(std::max<uint16_t>(to_u16(h, col[q]), c.p0 + 1), 65533);
    c.p75 = std::min<uint16_t>(std::max<uint16_t>(to_u16(h, col[3 * q]), c.p25 + 1), 65534);
    c.p100 = std::max<uint16_t>(to_u16(h, col[n - 1]), c.p75 + 1);
  } else {
    c.p0 = std::min<uint16_t>(to_u16(h, col[0]), 65532);
    c.p25 = n > 1 ? std::min<uint16_t>(std::max<uint16_t>(to_u16(h, col[1]), c.p0 + 1), 65533)
                  : (uint16_t)(c.p0 + 1);
    c.p75 = n > 2 ? std::min<uint16_t>(std::max<uint16_t>(to_u16(h, col[2]), c.p25 + 1), 65534)
                  : (uint16_t)(c.p25 + 1);
    c.p100 = n > 3 ? std::max<uint16_t>(to_u16(h, col[3]), c.p75 + 1) : (uint16_t)(c.p75 + 1);
  }
  return c;
}

std::vector<uint8_t> cm_compress(const float *m, int rows, int cols) {
  if (rows <= 0 || cols <= 0) return {};
  float mn = m[0], mx = m[0];
  for (long i = 0; i < (long)rows * cols; i++) {
    mn = std::min(mn, m[i]);
    mx = std::max(mx, m[i]);
  }
  if (mx == mn) mx = (float)((double)mn + (1.0 + (double)std::fabs(mn)));  // double, as the reference
  CmHeader h;
  h.min_value = mn;
  h.range = mx - mn;
  if (!std::isfinite(h.min_value) || !std::isfinite(h.range))
    throw std::invalid_argument("CompressedMatrix: matrix has inf or nan");
  if (h.range <= 0.0f) h.range = 1.0e-05f;
  h.num_rows = rows;
  h.num_cols = cols;
  h.format = rows > 8 ? 1 : 2;
  std::vector<uint8_t> out(sizeof(CmHeader) + cm_body_bytes(h));
  memcpy(out.data(), &h, sizeof(h));
  uint8_t *body = out.data() + sizeof(CmHeader);
  if (h.format == 1) {
    auto *hdr = reinterpret_cast<CmPerCol *>(body);
    uint8_t *bytes = body + sizeof(CmPerCol) * cols;
    std::vector<float> col(rows);
    for (int c = 0; c < cols; c++) {
      for (int r = 0; r < rows; r++) col[r] = m[(long)r * cols + c];
      const CmPerCol ph = col_header(h, col);
      memcpy(hdr + c, &ph, sizeof(ph));
      const float p0 = from_u16(h, ph.p0), p25 = from_u16(h, ph.p25), p75 = from_u16(h, ph.p75),
                  p100 = from_u16(h, ph.p100);
      for (int r = 0; r < rows; r++) bytes[(long)c * rows + r] = to_u8(p0, p25, p75, p100, m[(long)r * cols + c]);
    }
  } else {
    auto *d = reinterpret_cast<uint16_t *>(body);
    for (long i = 0; i < (long)rows * cols; i++) {
      const uint16_t v = to_u16(h, m[i]);
      memcpy(d + i, &v, 2);
    }
  }
  return out;
}

void cm_decompress(const uint8_t *data, float *out) {
  CmHeader h;
  memcpy(&h, data, sizeof(h));
  const uint8_t *body = data + sizeof(CmHeader);
  if (h.format == 1) {
    const uint8_t *bytes = body + sizeof(CmPerCol) * h.num_cols;
    for (int c = 0; c < h.num_cols; c++) {
      CmPerCol ph;
      memcpy(&ph, body + sizeof(CmPerCol) * c, sizeof(ph));
      const float p0 = from_u16(h, ph.p0), p25 = from_u16(h, ph.p25), p75 = from_u16(h, ph.p75),
                  p100 = from_u16(h, ph.p100);
      for (int r = 0; r < h.num_rows; r++)
        out[(long)r * h.num_cols + c] = from_u8(p0, p25, p75, p100, bytes[(long)c * h.num_rows + r]);
    }
  } else {
    for (long i = 0; i < (long)h.num_rows * h.num_cols; i++) {
      uint16_t v;
      memcpy(&v, body + 2 * i, 2);
      out[i] = from_u16(h, v);
    }
  }
}

int Example::NumFrames() const {
  if (cm.size() < sizeof(CmHeader)) return 0;
  CmHeader h;
  memcpy(&h, cm.data(), sizeof(h));
  return h.num_rows;
}
int Example::NumCols() const {
  if (cm.size() < sizeof(CmHeader)) return 0;
  CmHeader h;
  memcpy(&h, cm.data(), sizeof(h));
  return h.num_cols;
}

// ---------------------------------------------------------------------------
// Kaldi binary token stream (base/io-funcs.{h,cc}, io-funcs-inl.h)
// ---------------------------------------------------------------------------
static std::string strip_spec(const std::string &spec) {
  std::string s = spec;
  const auto colon = s.find(':');
  if (colon != std::string::npos) {
    std::string kind = s.substr(0, colon);
    // options like "ark,s,cs:" are accepted; scp is not supported here
    if (kind.compare(0, 3, "ark") != 0) throw std::invalid_argument("only ark: specifiers are supported: " + spec);
    s = s.substr(colon + 1);
  }
  return s;
}

namespace {
struct In {
  std::istream &is;
  [[noreturn]] void fail(const std::string &what) {
    throw std::runtime_error("egs archive: " + what + " at byte " + std::to_string((long long)is.tellg()));
  }
  std::string token() {  // ReadToken: non-space run, then one space
    std::string t;
    int c;
    while ((c = is.get()) != EOF && !isspace(c)) t.push_back((char)c);
    if (c == EOF && t.empty()) fail("unexpected end of stream");
    return t;
  }
  void expect(const char *tok) {
    const std::string t = token();
    if (t != tok) fail(std::string("expected token ") + tok + ", got " + t);
  }
  template <typename T>
  T basic() {  // ReadBasicType: size byte, then the raw integer
    const int sz = is.get();
    if (sz != (int)sizeof(T)) fail("bad integer size byte " + std::to_string(sz));
    T v;
    is.read(reinterpret_cast<char *>(&v), sizeof(T));
    if (!is) fail("short read");
    return v;
  }
  void raw(void *p, size_t n) {
    is.read(static_cast<char *>(p), (std::streamsize)n);
    if (!is) fail("short read");
  }
};

struct Out {
  std::ostream &os;
  void token(const char *t) { os << t << ' '; }
  template <typename T>
  void basic(T v) {
    os.put((char)sizeof(T));
    os.write(reinterpret_cast<const char *>(&v), sizeof(T));
  }
  void raw(const void *p, size_t n) { os.write(static_cast<const char *>(p), (std::streamsize)n); }
};
}  // namespace

// Matrix<float>::Read binary ("FM", or "DM" converted) -> compressed, as
// CompressedMatrix::Read does for an uncompressed matrix (compressed-matrix.cc:378-395)
static std::vector<uint8_t> read_plain_matrix(In &in, const std::string &tok) {
  const int rows = in.basic<int32_t>(), cols = in.basic<int32_t>();
  if (rows < 0 || cols < 0) in.fail("bad matrix size");
  std::vector<float> m((size_t)rows * cols);
  if (tok == "FM") {
    in.raw(m.data(), m.size() * 4);
  } else if (tok == "DM") {
    std::vector<double> dm(m.size());
    in.raw(dm.data(), dm.size() * 8);
    for (size_t i = 0; i < m.size(); i++) m[i] = (float)dm[i];
  } else {
    in.fail("expected CM, CM2, FM or DM, got " + tok);
  }
  return cm_compress(m.data(), rows, cols);
}

static void read_example(In &in, Example *eg) {
  in.expect("<NnetCtcExample>");
  in.expect("<Labels>");
  {
    const int sz = in.is.get();
    if (sz != 4) in.fail("labels: expected int32 vector");
    int32_t n;
    in.raw(&n, 4);
    if (n < 0) in.fail("labels: negative size");
    eg->labels.resize(n);
    if (n) in.raw(eg->labels.data(), 4 * (size_t)n);
  }
  in.expect("<InputFrames>");
  {
    const std::string tok = in.token();
    if (tok == "CM" || tok == "CM2") {
      CmHeader h;
      h.format = tok == "CM" ? 1 : 2;
      in.raw(reinterpret_cast<char *>(&h) + 4, sizeof(h) - 4);
      if (h.num_cols == 0 || h.num_rows == 0) {
        eg->cm.clear();
      } else {
        if (h.num_rows < 0 || h.num_cols < 0) in.fail("bad compressed matrix size");
        eg->cm.resize(sizeof(h) + cm_body_bytes(h));
        memcpy(eg->cm.data(), &h, sizeof(h));
        in.raw(eg->cm.data() + sizeof(h), cm_body_bytes(h));
      }
    } else {
      eg->cm = read_plain_matrix(in, tok);
    }
  }
  in.expect("<LeftContext>");
  eg->left_context = in.basic<int32_t>();
  in.expect("<SpkInfo>");
  {
    const std::string tok = in.token();
    const int32_t n = in.basic<int32_t>();
    if (n < 0) in.fail("spk_info: negative size");
    eg->spk_info.resize(n);
    if (tok == "FV") {
      if (n) in.raw(eg->spk_info.data(), 4 * (size_t)n);
    } else if (tok == "DV") {
      std::vector<double> v(n);
      if (n) in.raw(v.data(), 8 * (size_t)n);
      for (int i = 0; i < n; i++) eg->spk_info[i] = (float)v[i];
    } else {
      in.fail("spk_info: expected FV or DV, got " + tok);
    }
  }
  in.expect("</NnetCtcExample>");
}

ArchiveReader::ArchiveReader(const std::string &rspecifier) : path_(strip_spec(rspecifier)) {
  is_.open(path_, std::ios::binary);
  if (!is_) throw std::runtime_error("cannot open egs archive " + path_);
}

bool ArchiveReader::Next(Example *eg) {
  In in{is_};
  // key: up to the first space (archive format: "<key> <object>")
  std::string key;
  int c;
  while ((c = is_.get()) != EOF && isspace(c)) {
  }
  if (c == EOF) return false;
  key.push_back((char)c);
  while ((c = is_.get()) != EOF && c != ' ') key.push_back((char)c);
  if (c == EOF) in.fail("truncated archive after key " + key);
  // binary header "\0B" (InitKaldiInputStream)
  if (is_.peek() != '\0') in.fail("text-mode archives are not supported (key " + key + ")");
  is_.get();
  if (is_.get() != 'B') in.fail("bad binary header (key " + key + ")");
  eg->key = key;
  read_example(in, eg);
  return true;
}

ArchiveWriter::ArchiveWriter(const std::string &wspecifier) {
  const std::string path = strip_spec(wspecifier);
  os_.open(path, std::ios::binary | std::ios::trunc);
  if (!os_) throw std::runtime_error("cannot write egs archive " + path);
}

void ArchiveWriter::Write(const Example &eg) {
  if (eg.key.empty() || eg.key.find(' ') != std::string::npos) throw std::invalid_argument("bad archive key");
  Out o{os_};
  os_ << eg.key << ' ';
  os_.put('\0');
  os_.put('B');
  o.token("<NnetCtcExample>");
  o.token("<Labels>");
  os_.put((char)4);
  const int32_t n = (int32_t)eg.labels.size();
  o.raw(&n, 4);
  if (n) o.raw(eg.labels.data(), 4 * (size_t)n);
  o.token("<InputFrames>");
  if (eg.cm.empty()) {
    o.token("CM");
    CmHeader h{};
    o.raw(reinterpret_cast<const char *>(&h) + 4, sizeof(h) - 4);
  } else {
    CmHeader h;
    memcpy(&h, eg.cm.data(), sizeof(h));
    o.token(h.format == 1 ? "CM" : "CM2");
    o.raw(eg.cm.data() + 4, eg.cm.size() - 4);
  }
  o.token("<LeftContext>");
  o.basic<int32_t>(eg.left_context);
  o.token("<SpkInfo>");
  o.token("FV");
  o.basic<int32_t>((int32_t)eg.spk_info.size());
  if (!eg.spk_info.empty()) o.raw(eg.spk_info.data(), 4 * eg.spk_info.size());
  o.token("</NnetCtcExample>");
  if (!os_) throw std::runtime_error("egs archive write failed");
}

void ArchiveWriter::Close() {
  os_.flush();
  os_.close();
}

// ---------------------------------------------------------------------------
// minibatch packing (FormatNnetInput bookkeeping, ctc-nnet-update.cc:351-383)
// ---------------------------------------------------------------------------
Minibatch::~Minibatch() {
  if (done) {
    (void)hipEventSynchronize(done);
    (void)hipEventDestroy(done);
  }
}

std::unique_ptr<Minibatch> pack_minibatch(std::vector<Example> &egs, int nnet_left, int nnet_right) {
  if (egs.empty()) return nullptr;
  auto mb = std::make_unique<Minibatch>();
  const int num_splice = 1 + nnet_left + nnet_right;
  if (nnet_left < 0 || nnet_right < 0) throw std::invalid_argument("FormatNnetInput: negative context");
  mb->num_splice = num_splice;
  const Example &e0 = egs[0];
  if (e0.NumFrames() < num_splice) throw std::invalid_argument("FormatNnetInput: example shorter than the splice");
  mb->feat_dim = e0.NumCols();
  mb->spk_dim = (int)e0.spk_info.size();
  const int left_context = e0.left_context;
  if (left_context < nnet_left) throw std::invalid_argument("FormatNnetInput: left_context < nnet left context");
  const int ignore = left_context - nnet_left;
  const int N = (int)egs.size();
  mb->N = N;
  size_t off = align_up(sizeof(EgDesc) * N, 16);
  std::vector<EgDesc> desc(N);
  for (int n = 0; n < N; n++) {
    const Example &e = egs[n];
    if (e.NumCols() != mb->feat_dim || (int)e.spk_info.size() != mb->spk_dim)
      throw std::invalid_argument("FormatNnetInput: examples of different dimensions in one minibatch");
    const int frames = e.NumFrames() - num_splice - ignore + 1;
    if (frames < 0) throw std::invalid_argument("FormatNnetInput: example shorter than its left context");
    CmHeader h;
    memcpy(&h, e.cm.data(), sizeof(h));
    EgDesc &d = desc[n];
    memset(&d, 0, sizeof(d));
    d.format = h.format;
    d.rows = h.num_rows;
    d.cols = h.num_cols;
    d.min_value = h.min_value;
    d.range = h.range;
    d.first = ignore;
    d.frames = frames;
    d.off = (int64_t)off;
    off = align_up(off + e.cm.size() - sizeof(CmHeader), 16);
    d.spk_off = -1;
    if (mb->spk_dim) {
      d.spk_off = (int64_t)off;
      off = align_up(off + 4 * (size_t)mb->spk_dim, 16);
    }
    mb->T_max = std::max(mb->T_max, frames);
    mb->keys.push_back(e.key);
    mb->num_frames.push_back(frames);
    mb->label_lengths.push_back((int32_t)e.labels.size());
    mb->labels.insert(mb->labels.end(), e.labels.begin(), e.labels.end());
  }
  mb->blob.assign(off, 0);
  memcpy(mb->blob.data(), desc.data(), sizeof(EgDesc) * N);
  for (int n = 0; n < N; n++) {
    const Example &e = egs[n];
    memcpy(mb->blob.data() + desc[n].off, e.cm.data() + sizeof(CmHeader), e.cm.size() - sizeof(CmHeader));
    if (mb->spk_dim) memcpy(mb->blob.data() + desc[n].spk_off, e.spk_info.data(), 4 * (size_t)mb->spk_dim);
  }
  return mb;
}

// ---------------------------------------------------------------------------
// NnetCtcExampleBackgroundReader (ctc-nnet-train.cc:31-183)
// ---------------------------------------------------------------------------
static constexpr int kMaxLabelLength = 639;  // MAX_WARPCTC_LABEL_LENGTH (ctc-nnet-train.cc:26)

BackgroundReader::BackgroundReader(const std::string &rspecifier, int minibatch_size, int max_frames,
                                   int nnet_left, int nnet_right)
    : reader_(rspecifier), minibatch_size_(minibatch_size), max_frames_(max_frames), left_(nnet_left),
      right_(nnet_right) {
  if (minibatch_size <= 0) throw std::invalid_argument("minibatch_size must be > 0");
  thread_ = std::thread([this] { Run(); });
}

BackgroundReader::~BackgroundReader() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (thread_.joinable()) thread_.join();
}

void BackgroundReader::Run() {
  try {
    while (true) {
      std::vector<Example> egs;
      Example eg;
      while ((int)egs.size() < minibatch_size_ && reader_.Next(&eg)) {
        const int F = eg.NumFrames(), L = (int)eg.labels.size();
        if (F > max_frames_ || L > kMaxLabelLength || F < 2 * L + 1) {
          std::lock_guard<std::mutex> lk(mu_);
          skipped_++;
          continue;
        }
        egs.push_back(std::move(eg));
        eg = Example();
      }
      std::unique_ptr<Minibatch> mb = pack_minibatch(egs, left_, right_);
      const bool last = !mb;
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] { return !slot_full_ || stop_; });
      if (stop_) return;
      read_ += (long)egs.size();
      slot_ = std::move(mb);
      slot_full_ = true;
      lk.unlock();
      cv_.notify_all();
      if (last) return;
    }
  } catch (const std::exception &e) {
    std::lock_guard<std::mutex> lk(mu_);
    error_ = e.what();
    slot_.reset();
    slot_full_ = true;
    cv_.notify_all();
  }
}

std::unique_ptr<Minibatch> BackgroundReader::Next() {
  std::unique_lock<std::mutex> lk(mu_);
  if (finished_) return nullptr;
  cv_.wait(lk, [this] { return slot_full_; });
  if (!error_.empty()) {
    finished_ = true;
    throw std::runtime_error(error_);
  }
  std::unique_ptr<Minibatch> mb = std::move(slot_);
  slot_full_ = false;
  if (!mb) finished_ = true;
  lk.unlock();
  cv_.notify_all();
  return mb;
}

}  // namespace egs
}  // namespace kctc
