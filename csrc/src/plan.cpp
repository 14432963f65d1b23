#include "psoup/plan.hpp"

#include <cmath>

#include "psoup/common.hpp"

namespace psoup {

std::vector<float> generate_dm_list(float dm_start, float dm_end, double tsamp, double pulse_width_us,
                                    double fch1, double foff, int nchans, double tol) {
  std::vector<float> dms;
  // dedisp stores dt/f0/df in its plan as float32 and receives ti/tol as
  // float32 from peasoup's float CLI fields; widen only afterwards.
  tsamp = static_cast<float>(tsamp);
  fch1 = static_cast<float>(fch1);
  foff = static_cast<float>(foff);
  tol = static_cast<float>(tol);
  pulse_width_us = static_cast<float>(pulse_width_us);
  double dt = tsamp * 1e6;
  double f = (fch1 + ((nchans / 2) - 0.5) * foff) * 1e-3;
  double tol2 = tol * tol;
  double a = 8.3 * foff / (f * f * f);
  double a2 = a * a;
  double b2 = a2 * static_cast<double>(nchans * nchans / 16.0);
  double c = (dt * dt + pulse_width_us * pulse_width_us) * (tol2 - 1.0);
  dms.push_back(dm_start);
  // Guard against a non-advancing recurrence (degenerate inputs).
  const size_t max_trials = 10000000;
  while (dms.back() < dm_end) {
    double prev = dms.back();
    double prev2 = prev * prev;
    double k = c + tol2 * a2 * prev2;
    double dm = (b2 * prev + std::sqrt(-a2 * b2 * prev2 + (a2 + b2) * k)) / (a2 + b2);
    if (!(static_cast<float>(dm) > dms.back())) PSOUP_THROW("DM list recurrence did not advance at dm=" << prev);
    dms.push_back(static_cast<float>(dm));
    if (dms.size() > max_trials) PSOUP_THROW("DM list too long");
  }
  return dms;
}

std::vector<float> generate_delay_table(int nchans, double tsamp, double fch1, double foff) {
  std::vector<float> t(static_cast<size_t>(nchans));
  float f0 = static_cast<float>(fch1), df = static_cast<float>(foff), dt = static_cast<float>(tsamp);
  for (int c = 0; c < nchans; ++c) {
    float a = 1.f / (f0 + c * df);
    float b = 1.f / f0;
    t[c] = static_cast<float>(4.15e3 / dt * (a * a - b * b));
  }
  return t;
}

int compute_max_delay(const std::vector<float>& dm_list, const std::vector<float>& delay_table) {
  if (dm_list.empty() || delay_table.empty()) return 0;
  float dmax = dm_list.back();
  float dl = delay_table.back();
  // foff > 0 puts the largest |delay| at channel 0; take the max magnitude.
  for (float d : delay_table)
    if (std::fabs(d) > std::fabs(dl)) dl = d;
  return dm_delay_samples(dmax, dl);
}

AccelPlan::AccelPlan(float acc_lo, float acc_hi, float tol, float pulse_width, uint64_t nsamps, float tsamp,
                     float cfreq, float bw, AccelConvention conv)
    : acc_lo_(acc_lo),
      acc_hi_(acc_hi),
      tol_(tol),
      pulse_width_(pulse_width),
      tsamp_(tsamp),
      cfreq_(cfreq),
      bw_(std::fabs(bw)),
      conv_(conv) {
  tobs_ = static_cast<float>(static_cast<float>(nsamps) * tsamp);
  if (conv_ == AccelConvention::Reference) pulse_width_ = static_cast<float>(pulse_width_ / 1.0e3);
}

float AccelPlan::step(float dm) const {
  float tdm = static_cast<float>(std::pow(8.3 * bw_ / std::pow(static_cast<double>(cfreq_), 3.0) * dm, 2.0));
  float tpulse = pulse_width_ * pulse_width_;
  float ttsamp = tsamp_ * tsamp_;
  float w_us = std::sqrt(tdm + tpulse + ttsamp);
  double alt = 2.0 * w_us * 1.0e-6 * 24.0 * 299792458.0 / tobs_ / tobs_ * std::sqrt(static_cast<double>(tol_ * tol_) - 1.0);
  return static_cast<float>(alt);
}

std::vector<float> AccelPlan::generate(float dm) const {
  std::vector<float> list;
  if (acc_hi_ == acc_lo_) {
    list.push_back(0.f);
    return list;
  }
  float alt_a = step(dm);
  PSOUP_CHECK(alt_a > 0.f && std::isfinite(alt_a), "non-positive acceleration step");
  if (acc_hi_ != 0.f && acc_lo_ != 0.f) list.push_back(0.f);
  float acc = acc_lo_;
  while (acc < acc_hi_) {
    list.push_back(acc);
    acc += alt_a;
    PSOUP_CHECK(list.size() < 50000000, "acceleration list too long");
  }
  list.push_back(acc_hi_);
  return list;
}

AccelConvention parse_accel_convention(const std::string& s) {
  if (s == "legacy" || s == "intended" || s == "golden") return AccelConvention::Legacy;
  if (s == "reference" || s == "current") return AccelConvention::Reference;
  PSOUP_THROW("unknown acceleration-plan convention '" << s << "' (legacy|reference)");
}

const char* accel_convention_name(AccelConvention c) {
  return c == AccelConvention::Legacy ? "legacy" : "reference";
}

}  // namespace psoup
