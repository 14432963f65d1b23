// Search plans: DM trial list, dispersion delay table, acceleration plan.
//
// Parity:
//  * DM list: external dedisp `dedisp_generate_dm_list` (called from
//    include/transforms/dedisperser.hpp:54-62) -- Lina Levin's algorithm in
//    double precision, stored as float32.  Reproduces the 59 trials of
//    example_output/overview.xml:63-123 bit-for-bit.
//  * Delay table: dedisp `generate_delay_table`:
//        delay[c] = 4.15e3/tsamp * (1/(fch1+c*foff)^2 - 1/fch1^2)   (float)
//    per-sample offset = (int)(dm*delay[c] + 0.5);
//    max_delay = (int)(dm_max*delay[nchans-1] + 0.5)  (dedisperser.hpp:100).
//  * Acceleration plan: include/utils/utils.hpp:140-193 AccelerationPlan.
//    The reference divides the pulse width by 1e3 (utils.hpp:165) while the
//    step formula treats it as microseconds, making the step 1000x finer than
//    intended.  AccelConvention::Legacy (the default here)
//    is the intended / golden-output behaviour (3 trials for tutorial.fil at
//    +-5 m/s^2); AccelConvention::Reference reproduces the current code.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace psoup {

std::vector<float> generate_dm_list(float dm_start, float dm_end, double tsamp, double pulse_width_us,
                                    double fch1, double foff, int nchans, double tol);

std::vector<float> generate_delay_table(int nchans, double tsamp, double fch1, double foff);

// Integer sample offset of channel c at DM `dm` (round half up, as dedisp).
inline int dm_delay_samples(float dm, float delay) { return static_cast<int>(dm * delay + 0.5f); }

int compute_max_delay(const std::vector<float>& dm_list, const std::vector<float>& delay_table);

enum class AccelConvention { Legacy = 0, Reference = 1 };

class AccelPlan {
 public:
  AccelPlan() = default;
  // Argument order and meaning as AccelerationPlan(acc_lo, acc_hi, tol,
  // pulse_width[us], nsamps(=fft size), tsamp, cfreq, bw) -- note that the
  // reference pipeline passes foff as `bw` (pipeline_multi.cu:335-337).
  AccelPlan(float acc_lo, float acc_hi, float tol, float pulse_width, uint64_t nsamps, float tsamp,
            float cfreq, float bw, AccelConvention conv = AccelConvention::Legacy);
  std::vector<float> generate(float dm) const;
  float step(float dm) const;
  float acc_lo() const { return acc_lo_; }
  float acc_hi() const { return acc_hi_; }
  AccelConvention convention() const { return conv_; }

 private:
  float acc_lo_ = 0.f, acc_hi_ = 0.f, tol_ = 1.1f, pulse_width_ = 64.f;
  float tsamp_ = 0.f, cfreq_ = 0.f, bw_ = 0.f, tobs_ = 0.f;
  AccelConvention conv_ = AccelConvention::Legacy;
};

AccelConvention parse_accel_convention(const std::string& s);
const char* accel_convention_name(AccelConvention c);

}  // namespace psoup
