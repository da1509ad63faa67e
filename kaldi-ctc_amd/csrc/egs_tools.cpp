// egs_tools.cpp -- the egs preparation tools that decide minibatch length
// homogeneity: nnet-ctc-shuffle-egs and nnet-ctc-sort-egs.
//
//   nnet-ctc-shuffle-egs        src/ctcbin/nnet-ctc-shuffle-egs.cc:25-127
//   nnet-ctc-sort-egs           src/ctcbin/nnet-ctc-sort-egs.cc:27-133
//   FrameSubsamplingShift...    src/ctc/ctc-nnet-example.cc:78-106
//
// The example order is the reference's exactly: the tools seed glibc's
// generator (srand) and draw with rand() through Kaldi's RandInt
// (base/kaldi-math.cc:100-127) and libstdc++'s std::random_shuffle
// (bits/stl_algo.h: j = rand() % (i + 1) for i = 1..n-1).  The same additive
// feedback generator is run here on a private state (initstate_r / random_r,
// the reentrant form of srand / rand: identical sequence) so the library does
// not disturb the host process's global rand() stream.  Sorting uses
// std::sort with the reference's comparator, so ties between equal lengths
// land in the same (implementation-defined) order as the reference binary
// built with g++.
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <memory>
#include <stdexcept>
#include <vector>

#include "egs.h"
#include "glibc_rand.h"

namespace kctc {
namespace egs {


void FrameSubsamplingShift(int frame_subsampling_factor, int frame_shift, Example *eg) {
  if (frame_subsampling_factor <= 1) return;
  if (!(frame_shift >= 0 && frame_shift < frame_subsampling_factor))
    throw std::invalid_argument("frame_shift must be in [0, frame_subsampling_factor)");
  const int rows = eg->NumFrames(), cols = eg->NumCols();
  if (rows == 0 || cols == 0) return;
  // Matrix full_src(eg->input_frames): decode
  std::vector<float> full((size_t)rows * cols);
  cm_decompress(eg->cm.data(), full.data());
  // rows frame_shift, frame_shift + f, ... (ctc-nnet-example.cc:83-86)
  std::vector<float> sel;
  int n = 0;
  for (int i = 0; i + frame_shift < rows; i += frame_subsampling_factor, n++)
    sel.insert(sel.end(), full.begin() + (size_t)(i + frame_shift) * cols,
               full.begin() + (size_t)(i + frame_shift + 1) * cols);
  // eg->input_frames = full_src re-compresses, even when no row was selected
  // (the matrix is then left as decoded, :87-88)
  eg->cm = n ? cm_compress(sel.data(), n, cols) : cm_compress(full.data(), rows, cols);
}

static std::vector<Example> read_all(const std::string &rspecifier) {
  ArchiveReader reader(rspecifier);
  std::vector<Example> egs;
  Example eg;
  while (reader.Next(&eg)) egs.push_back(std::move(eg));
  return egs;
}

long ShuffleEgs(const std::string &rspecifier, const std::string &wspecifier, int srand_seed,
                int buffer_size, int frame_shift, int frame_subsampling_factor) {
  if (buffer_size < 0) throw std::invalid_argument("buffer_size must be >= 0");
  GlibcRand rng((unsigned)srand_seed);
  ArchiveWriter writer(wspecifier);
  long num_done = 0;
  std::vector<std::unique_ptr<Example>> egs;
  if (buffer_size == 0) {  // full randomization (:79-87)
    for (auto &e : read_all(rspecifier)) egs.emplace_back(new Example(std::move(e)));
    for (size_t i = 1; i < egs.size(); i++) {  // std::random_shuffle
      const size_t j = (size_t)rng() % (i + 1);
      if (i != j) std::swap(egs[i], egs[j]);
    }
  } else {  // limited-memory partial randomization (:88-106)
    egs.resize(buffer_size);
    ArchiveReader reader(rspecifier);
    Example eg;
    while (reader.Next(&eg)) {
      const int index = rng.RandInt(0, buffer_size - 1);
      if (!egs[index]) {
        egs[index].reset(new Example(std::move(eg)));
      } else {
        if (frame_subsampling_factor > 0)
          FrameSubsamplingShift(frame_subsampling_factor, frame_shift, egs[index].get());
        writer.Write(*egs[index]);
        *egs[index] = std::move(eg);
        num_done++;
      }
      eg = Example();
    }
  }
  for (auto &e : egs) {  // (:107-115)
    if (!e) continue;
    if (frame_subsampling_factor > 1) FrameSubsamplingShift(frame_subsampling_factor, frame_shift, e.get());
    writer.Write(*e);
    num_done++;
  }
  writer.Close();
  return num_done;
}

long SortEgs(const std::string &rspecifier, const std::string &wspecifier, int srand_seed,
             int buffer_size) {
  (void)srand_seed;  // seeded by the reference tool, but never drawn from
  if (buffer_size < 0) throw std::invalid_argument("buffer_size must be >= 0");
  ArchiveWriter writer(wspecifier);
  // SortNnetCtcExample (:29-32): by NumFrames, std::sort (not stable)
  auto by_frames = [](const std::unique_ptr<Example> &a, const std::unique_ptr<Example> &b) {
    return a->NumFrames() < b->NumFrames();
  };
  long num_done = 0;
  size_t num_read = 0;
  std::vector<std::unique_ptr<Example>> egs;
  if (buffer_size == 0) {  // full sort (:76-84)
    for (auto &e : read_all(rspecifier)) egs.emplace_back(new Example(std::move(e)));
    std::sort(egs.begin(), egs.end(), by_frames);
    num_read = egs.size();
  } else {  // partial sort (:85-108): a full buffer is sorted and written when
            // the NEXT example arrives, so the last buffer's worth (1..buffer_size
            // examples) is written in arrival order, unsorted, as the reference does
    egs.resize(buffer_size);
    ArchiveReader reader(rspecifier);
    Example eg;
    while (reader.Next(&eg)) {
      if (num_read > 0 && num_read % (size_t)buffer_size == 0) {
        std::sort(egs.begin(), egs.end(), by_frames);
        for (auto &e : egs) {
          writer.Write(*e);
          num_done++;
        }
        num_read = 0;
      }
      if (!egs[num_read])
        egs[num_read].reset(new Example(std::move(eg)));
      else
        *egs[num_read] = std::move(eg);
      eg = Example();
      num_read++;
    }
  }
  for (size_t i = 0; i < egs.size() && i < num_read; i++) {  // (:110-118)
    writer.Write(*egs[i]);
    num_done++;
  }
  writer.Close();
  return num_done;
}

}  // namespace egs
}  // namespace kctc
