// glibc_rand.h -- the host process's rand() stream of the reference tools,
// on a private state.
//
// The reference seeds glibc's generator once per process (srand(--srand),
// e.g. src/ctcbin/nnet2-ctc-train-simple.cc:47,69) and every later draw goes
// through kaldi::Rand() -> rand() (src/base/kaldi-math.cc:46-62):
//   RandInt(lo, hi)  lo + rand() % (hi + 1 - lo), no draw when hi == lo
//                    (kaldi-math.cc:100-127)
//   RandUniform()    (float)((rand() + 1.0) / (RAND_MAX + 2.0))
//                    (src/base/kaldi-math.h:151-153)
// glibc's own reentrant form (initstate_r / random_r on a 128-byte TYPE_3
// state, the default generator behind srand / rand) gives the identical
// sequence without touching the host process's global stream.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace kctc {

class GlibcRand {
 public:
  explicit GlibcRand(unsigned seed = 0) { Seed(seed); }
  GlibcRand(const GlibcRand &) = delete;
  GlibcRand &operator=(const GlibcRand &) = delete;
  void Seed(unsigned seed) {  // srand(seed)
    memset(&rd_, 0, sizeof(rd_));
    memset(state_, 0, sizeof(state_));
    if (initstate_r(seed, state_, sizeof(state_), &rd_) != 0) throw std::runtime_error("initstate_r failed");
    calls_ = 0;
  }
  int operator()() {  // rand()
    int32_t r = 0;
    random_r(&rd_, &r);
    calls_++;
    return (int)r;
  }
  int RandInt(int lo, int hi) {
    if (hi == lo) return lo;
    return lo + ((*this)() % (hi + 1 - lo));
  }
  float RandUniform() { return static_cast<float>(((*this)() + 1.0) / (RAND_MAX + 2.0)); }
  long Calls() const { return calls_; }

 private:
  char state_[128];
  struct random_data rd_;
  long calls_ = 0;
};

}  // namespace kctc
