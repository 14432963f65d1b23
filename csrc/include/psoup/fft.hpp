// rocFFT plan wrapper (replaces include/transforms/ffter.hpp:7-78, the cuFFT
// cufftPlan1d R2C/C2R/C2C wrappers).  Plans are batched, carry their own work
// area, and execute asynchronously on the caller's stream.  Transforms are
// unnormalised in both directions (cuFFT semantics).
#pragma once

#include <hip/hip_runtime.h>
#include <rocfft/rocfft.h>

#include <cstdint>
#include <memory>

#include "psoup/common.hpp"

namespace psoup {

enum class FftType { R2C, C2R, C2C_FWD, C2C_INV };

class FftPlan {
 public:
  // in_dist / out_dist: element distance between batch members (0 = packed);
  // in_stride / out_stride: element distance within one transform.
  FftPlan(FftType type, uint64_t n, uint64_t batch = 1, uint64_t in_dist = 0, uint64_t out_dist = 0,
          bool inplace = false, uint64_t in_stride = 1, uint64_t out_stride = 1);
  ~FftPlan();
  FftPlan(const FftPlan&) = delete;
  FftPlan& operator=(const FftPlan&) = delete;

  void execute(void* in, void* out, hipStream_t stream);
  uint64_t n() const { return n_; }
  uint64_t batch() const { return batch_; }
  FftType type() const { return type_; }
  size_t work_bytes() const { return work_.bytes(); }

 private:
  FftType type_;
  uint64_t n_, batch_;
  bool inplace_;
  rocfft_plan plan_ = nullptr;
  rocfft_execution_info info_ = nullptr;
  DeviceBuffer<uint8_t> work_;
};

// Resolution of an N-point transform: 1/(N*tsamp)  (ffter.hpp:21-23)
inline double fft_resolution(uint64_t n, float tsamp) { return 1.0 / (static_cast<double>(n) * tsamp); }

void fft_global_setup();

}  // namespace psoup
