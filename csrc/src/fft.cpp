#include "psoup/fft.hpp"

#include <mutex>

namespace psoup {

#define PSOUP_ROCFFT_CHECK(expr)                                        \
  do {                                                                  \
    rocfft_status _st = (expr);                                         \
    if (_st != rocfft_status_success)                                   \
      PSOUP_THROW("rocFFT error " << static_cast<int>(_st) << " in " #expr); \
  } while (0)

void fft_global_setup() {
  static std::once_flag once;
  std::call_once(once, [] { PSOUP_ROCFFT_CHECK(rocfft_setup()); });
}

FftPlan::FftPlan(FftType type, uint64_t n, uint64_t batch, uint64_t in_dist, uint64_t out_dist, bool inplace,
                 uint64_t in_stride, uint64_t out_stride)
    : type_(type), n_(n), batch_(batch), inplace_(inplace) {
  PSOUP_CHECK(n >= 1 && batch >= 1 && in_stride >= 1 && out_stride >= 1, "bad FFT size");
  fft_global_setup();
  rocfft_transform_type tt;
  rocfft_array_type ain, aout;
  uint64_t in_len, out_len;
  switch (type) {
    case FftType::R2C:
      tt = rocfft_transform_type_real_forward;
      ain = rocfft_array_type_real;
      aout = rocfft_array_type_hermitian_interleaved;
      in_len = n;
      out_len = n / 2 + 1;
      break;
    case FftType::C2R:
      tt = rocfft_transform_type_real_inverse;
      ain = rocfft_array_type_hermitian_interleaved;
      aout = rocfft_array_type_real;
      in_len = n / 2 + 1;
      out_len = n;
      break;
    case FftType::C2C_FWD:
      tt = rocfft_transform_type_complex_forward;
      ain = aout = rocfft_array_type_complex_interleaved;
      in_len = out_len = n;
      break;
    default:
      tt = rocfft_transform_type_complex_inverse;
      ain = aout = rocfft_array_type_complex_interleaved;
      in_len = out_len = n;
      break;
  }
  if (in_dist == 0) in_dist = in_len;
  if (out_dist == 0) out_dist = out_len;
  if (inplace && (type == FftType::R2C || type == FftType::C2R)) {
    // in-place real transforms need padded real rows of 2*(n/2+1)
    if (type == FftType::R2C) in_dist = 2 * (n / 2 + 1);
    else out_dist = 2 * (n / 2 + 1);
  }
  rocfft_plan_description desc = nullptr;
  PSOUP_ROCFFT_CHECK(rocfft_plan_description_create(&desc));
  size_t istride = static_cast<size_t>(in_stride), ostride = static_cast<size_t>(out_stride);
  size_t lengths[1] = {static_cast<size_t>(n)};
  rocfft_status st = rocfft_plan_description_set_data_layout(desc, ain, aout, nullptr, nullptr, 1, &istride,
                                                             static_cast<size_t>(in_dist), 1, &ostride,
                                                             static_cast<size_t>(out_dist));
  if (st != rocfft_status_success) {
    rocfft_plan_description_destroy(desc);
    PSOUP_THROW("rocfft_plan_description_set_data_layout failed: " << static_cast<int>(st));
  }
  st = rocfft_plan_create(&plan_, inplace ? rocfft_placement_inplace : rocfft_placement_notinplace, tt,
                          rocfft_precision_single, 1, lengths, static_cast<size_t>(batch), desc);
  rocfft_plan_description_destroy(desc);
  if (st != rocfft_status_success)
    PSOUP_THROW("rocfft_plan_create failed (" << static_cast<int>(st) << ") for n=" << n << " batch=" << batch);
  size_t wbytes = 0;
  PSOUP_ROCFFT_CHECK(rocfft_plan_get_work_buffer_size(plan_, &wbytes));
  PSOUP_ROCFFT_CHECK(rocfft_execution_info_create(&info_));
  if (wbytes > 0) {
    work_.resize(wbytes);
    PSOUP_ROCFFT_CHECK(rocfft_execution_info_set_work_buffer(info_, work_.data(), wbytes));
  }
}

FftPlan::~FftPlan() {
  if (info_) rocfft_execution_info_destroy(info_);
  if (plan_) rocfft_plan_destroy(plan_);
}

void FftPlan::execute(void* in, void* out, hipStream_t stream) {
  PSOUP_ROCFFT_CHECK(rocfft_execution_info_set_stream(info_, stream));
  void* ib[1] = {in};
  void* ob[1] = {out};
  PSOUP_ROCFFT_CHECK(rocfft_execute(plan_, ib, inplace_ ? nullptr : ob, info_));
  post_launch_check("rocfft_execute", stream);
}

}  // namespace psoup
