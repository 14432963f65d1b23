// Per-GPU engine: resident filterbank, dedispersion, whitening, batched
// acceleration search, candidate folding, coincidence masks.
//
// Parity (reference -> here):
//   Dedisperser (dedisperser.hpp:12-114, external dedisp)  -> DeviceFilterbank + Dedisperser
//   Worker::start (pipeline_multi.cu:100-252), one accel trial at a time with a
//     device sync after every kernel                       -> SearchEngine::search_trial
//     (whitening fused into 5 kernels; K accelerations per batched rocFFT;
//      fused harmonic-sum/peak kernel; peak lists copied on a second stream
//      while the next batch computes; host clustering/distillation overlapped)
//   Dereddener/Zapper/SpectrumFormer                       -> Whitener
//   MultiFolder/TimeSeriesFolder/FoldOptimiser (folder.hpp) -> FoldEngine
//   Coincidencer (coincidencer.hpp)                         -> beam_indicator + coincidence
#pragma once

#include <hip/hip_runtime.h>

#include <functional>
#include <deque>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "psoup/candidates.hpp"
#include "psoup/common.hpp"
#include "psoup/fft.hpp"
#include "psoup/kernels.hpp"
#include "psoup/plan.hpp"
#include "psoup/sigproc.hpp"

namespace psoup {

// Valu: the byte kernels (LDS-staged or global); Packed2: the 2-bit kernel
// (nbits <= 2 only); Auto: LDS-fed MFMA on the narrow-spread leading tiles,
// then Packed2 where the data allows, else Valu.
enum class DedispKernel { Auto = 0, Direct = 1, Mfma = 2, Valu = 3, Packed2 = 4 };
DedispKernel parse_dedisp_kernel(const std::string& s);

// Geometry shared by every rank: DM list, delays, killmask, output length.
struct DedispGeometry {
  int nchans = 0;
  int nbits = 0;
  double tsamp = 0, fch1 = 0, foff = 0;
  uint64_t nsamps = 0;
  std::vector<float> dm_list;
  std::vector<float> delays;
  std::vector<int> killmask;
  int max_delay = 0;
  uint64_t out_nsamps = 0;
  float out_scale = 1.f;
  int bias = 0;
  int nactive = 0;
  static DedispGeometry make(const SigprocHeader& hdr, uint64_t nsamps, const std::vector<float>& dm_list,
                             const std::vector<int>& killmask);
  // int32 [ndm][nchans] sample offsets for DMs [d0, d1)
  std::vector<int32_t> offsets(int d0, int d1) const;
};

// Channel-major int8 filterbank resident in HBM.
class DeviceFilterbank {
 public:
  DeviceFilterbank(const DedispGeometry& g, hipStream_t stream);
  // Packed (SIGPROC layout) bytes already on this device (e.g. after an RCCL broadcast).
  void load_packed_device(const uint8_t* d_packed);
  // Packed bytes in host memory (H2D in chunks through pinned staging).
  void load_packed_host(const uint8_t* h_packed);
  // Samples [t0, t0 + ns) from their packed bytes on this device (stream s;
  // nullptr = the constructor's stream).
  void unpack_chunk(const uint8_t* d_packed, uint64_t t0, uint64_t ns, hipStream_t s = nullptr);
  hipStream_t stream() const { return stream_; }
  const int8_t* data() const { return chan_.data(); }
  uint64_t stride() const { return stride_; }
  // narrow data (nbits <= 2): the rows again as 2-bit fields, 16 samples per
  // dword (kern::pack2_rows), zero-padded past the int8 rows; else nullptr
  const uint32_t* data2() const { return chan2_.size() ? chan2_.data() : nullptr; }
  uint64_t stride2() const { return stride2_; }
  const DedispGeometry& geometry() const { return g_; }

 private:
  void pack2(uint64_t t0, uint64_t ns, hipStream_t s);
  DedispGeometry g_;
  hipStream_t stream_;
  uint64_t stride_, stride2_ = 0;
  DeviceBuffer<int8_t> chan_;
  DeviceBuffer<uint32_t> chan2_;
};

// One host upload, then a device-to-device fan-out (SURVEY.md §2.7, §5.8
// item 1): the packed filterbank goes host -> devs[0] in chunks through pinned
// staging; every other device copies each chunk from devs[0] as it lands
// (hipMemcpyPeerAsync: SDMA over xGMI, all peers in parallel on their own
// links) and unpacks it while the next chunk is in flight.  fbs[i] lives on
// HIP device devices[i] (the same device may repeat: a device-local copy).
// Returns when every device holds its unpacked filterbank.
// (read(off, n, dst): host bytes [off, off + n) of the packed data into dst)
using HostReader = std::function<void(uint64_t, uint64_t, uint8_t*)>;
void load_filterbank_fanout(const std::vector<DeviceFilterbank*>& fbs, const std::vector<int>& devices,
                            const HostReader& read);
void load_filterbank_fanout(const std::vector<DeviceFilterbank*>& fbs, const std::vector<int>& devices,
                            const uint8_t* h_packed);
// straight from the file (threaded pread into the pinned stages)
void load_filterbank_fanout(const std::vector<DeviceFilterbank*>& fbs, const std::vector<int>& devices,
                            const Filterbank& fb);
// Host bytes [0, bytes) -> d_dst on stream s in `chunk`-byte pieces through two
// pinned stages filled by `read` (chunk k+1 is read while chunk k copies);
// on_chunk(off, n) runs after each piece's copy is enqueued.  Returns when the
// stages are free (the copies done).
void staged_upload(uint64_t bytes, uint64_t chunk, const HostReader& read, uint8_t* d_dst, hipStream_t s,
                   const std::function<void(uint64_t, uint64_t)>& on_chunk = {});

class Dedisperser {
 public:
  Dedisperser(const DeviceFilterbank& fb, hipStream_t stream);
  // DM trials [d0, d1) -> out[(d-d0)*out_stride + t], t < out_nsamps, on
  // stream s (nullptr = the constructor's stream).  MFMA runs made of whole
  // Every range (tile-aligned or not) runs on the resident tables (built on
  // first use or by warm(), one upload each) and never blocks the host; a
  // range not starting on a tile computes its first tile (or workgroup) whole
  // and stores from d0.
  void run(int d0, int d1, uint8_t* out, uint64_t out_stride, DedispKernel kind = DedispKernel::Auto,
           hipStream_t s = nullptr);
  // An arbitrary list of DM indices (row i = DM dms[i]) in ONE packed-byte
  // VALU launch over ceil(n / 32) DM tiles (the fold stage: scattered DMs,
  // where per-DM runs would each pay a whole tile).  Bit-identical to run().
  // Waits for its offset-table upload (the host table goes out of scope);
  // successive calls must share one stream (the device table is reused).
  void run_list(const std::vector<int>& dms, uint8_t* out, uint64_t out_stride, hipStream_t s = nullptr);
  static uint64_t row_stride(uint64_t out_nsamps) { return (out_nsamps + 255) / 256 * 256; }
  static constexpr int kTileDms = 32;  // DMs per MFMA tile
  // Auto's choice for [d0, d1): one-hot MFMA while the tiles' offset spread is
  // narrow (few 16-shift blocks per channel), packed-byte VALU once it is wide.
  DedispKernel choose(int d0, int d1);
  // global-load MFMA steps per (tile, active channel) over [d0, d1)'s tiles
  double mfma_steps_per_channel(int d0, int d1);
  // Auto's split of a tile-aligned range: DMs [d0, split) run the LDS-fed
  // MFMA kernel (leading tiles whose offset spread is narrow enough for the
  // one-hot GEMM to beat the VALU kernels), [split, d1) the VALU kernels
  int mfma_lds_split(int d0, int d1);
  // Build the tables Auto / MFMA / VALU runs use over DMs [d0, d1) (d1 < 0:
  // the whole list; a static shard needs only its own).  Otherwise they are
  // built on the first run that needs them, with blocking uploads,
  // mid-search (the 2026-DM config-4 list's first VALU tile stalled the host
  // 64 ms); a run outside the built tiles rebuilds the whole list's.
  void warm(int d0 = 0, int d1 = -1);

 private:
  void build_resident_plan();
  void ensure_tables(int d0, int d1);
  void build_tables(int t0, int t1);  // tiles [t0, t1)
  // offs: rows of DMs [e0, ...) covering tiles [t0, t1 + 1)
  void build_valu_tables(const std::vector<int32_t>& offs, int e0, int t0, int t1);
  int max_spread(int d0, int d1) const;  // largest (offset - window start) over [d0, d1)'s tiles
  void upload_mfma_lds_tables(const kern::MfmaLdsPlan& plan);
  void run_mfma_lds(int d0, int d1, uint8_t* out, uint64_t out_stride, hipStream_t s);
  const DeviceFilterbank& fb_;
  hipStream_t stream_;
  DeviceBuffer<int32_t> d_offsets_, d_kill_, d_active_, d_list_offT_;
  bool resident_ = false;
  int tab_t0_ = 0, tab_t1_ = 0;  // tiles the VALU and LDS-MFMA tables cover
  std::vector<int32_t> h_tile_steps_;  // global-load MFMA plan's steps per tile (from the VALU tables)
  int ldo_ = 0;                        // columns of r_offT_
  std::vector<int32_t> h_tile_win_;    // LDS kernel: largest channel window per 32-DM tile (bytes)
  DeviceBuffer<int32_t> r_steps_, r_tile_info_, r_offT_, r_wmin_;
  DeviceBuffer<int8_t> r_deltas_;
  // LDS-fed MFMA plan (tiles [tab_t0_, tab_t1_) built, the others not-ok)
  int ml_ngroups_ = 0;
  std::vector<int32_t> ml_tile_ok_, ml_tile_steps_;
  DeviceBuffer<int32_t> ml_steps_, ml_ginfo_, ml_wmin_;
  DeviceBuffer<uint8_t> ml_relo_;
};

struct SearchParams {
  uint64_t fft_size = 0;
  float tsamp = 0.f;
  float min_snr = 9.f;
  float min_freq = 0.1f;
  float max_freq = 1100.f;
  int nharmonics = 4;
  float freq_tol = 0.0001f;
  int max_harm = 16;
  float boundary_5_freq = 0.05f;
  float boundary_25_freq = 0.5f;
  std::vector<float> zap_freqs, zap_widths;
  int accel_batch = 0;          // 0 = auto
  int sub_batch = -1;           // fused-FFT trials per sub-batch on alternating streams (0 = off, -1 = auto)
  int host_threads = -1;        // host workers clustering/distilling peak-heavy batches (-1 = auto, 0/1 = serial)
  // auto-batch HBM budget (2048 trials of 2^23: 112 GB of intermediates --
  // Y, P, Q -- on a 288 GB device; same-box sweep of the round-5 bench with
  // the non-temporal Y / P stores: K = 2048 36.23k/36.19k, 1536
  // 36.15k/36.13k, 1024 35.81k/35.67k, 768 35.84k/35.89k trials/s,
  // profiles/r5_batch/), capped at 70% of the device's free memory shared
  // among its engines
  size_t batch_bytes = 128ull << 30;
  // Engines sharing the device: the auto budget is also capped at 70% of the
  // device's free memory divided by this count.
  int engines_per_device = 1;
  // Auto batching of short trial lists: lists shorter than min_batches full
  // batches are cut into min_batches even batches (multiples of 8), but never
  // below the batch an eighth of the budget gives.
  // (4: the bench's 8-DM lists of 5480 trials at 2^23 run as 4 x 1376; 3 x
  // 1832 was 0.6% faster on noise but put peak-heavy data below 90% of it)
  int min_batches = 4;
  // Threshold-crossing records in 2^peak_region_log2 regions with a counter
  // each (kern::kPeakRegionStride) when the device clusters them: the
  // reservation atomics of peak-heavy batches spread over that many lines.
  int peak_region_log2 = 6;
  // Compute streams the sub-batches of a batch rotate over (>= 2).
  int sub_streams = 2;
  int min_gap = 30;
  // Acceleration-trial FFT path: 0 = rocFFT R2C of N points; 1 = rocFFT C2C
  // of N/2 points with the real-FFT post-processing fused into the interbin
  // kernel; 2 = resample fused into a two-pass four-step FFT (fft4step.hip,
  // default; falls back to 1 when N/2 is not N1*N2 with N1,N2 in 128..4096).
  int fft_mode = 2;
};

// Running-median whitening of one N-point series, in place.
class Whitener {
 public:
  // allow_fft4: run the N-point real transforms on the four-step FFT passes
  // (K = 1) when the geometry allows; otherwise (or when false) rocFFT.
  Whitener(uint64_t n, float tsamp, hipStream_t stream, bool allow_fft4 = true);
  // trial u8[nsamps] -> d_series f32[n] (pad with mean / truncate)
  void load_trial(const uint8_t* d_trial, uint64_t nsamps, float* d_series);
  // R2C, running median, deredden (+zap), [interbin stats], C2R in place.
  void whiten(float* d_series, const uint32_t* d_zapmask, bool with_stats, float boundary5, float boundary25);
  // load_trial + whiten (with stats) for `count` trials in one batch: trial b
  // at d_trials + b*row_stride -> d_out + b*out_stride, its interbin stats
  // {mean, rms, std} at d_stats + 4b.  The forward and inverse transforms run
  // as one K = count four-step FFT each (rocFFT per trial without fft4).
  // With pad_out (and its geometry pad_g), the whitened series may instead be
  // written straight into pass A's padded row input, trial b at pad_out +
  // b*pad_stride (fft4_c2r_post_pad); the return value says whether it was,
  // in which case d_out is left unwritten.
  bool whiten_batch(const uint8_t* d_trials, uint64_t row_stride, uint64_t nsamps, int count, float* d_out,
                    uint64_t out_stride, const uint32_t* d_zapmask, float* d_stats, float boundary5,
                    float boundary25, float* pad_out = nullptr, const kern::Fft4Geom* pad_g = nullptr,
                    uint64_t pad_stride = 0);
  // device bytes whiten_batch holds per trial of its largest batch
  uint64_t batch_bytes_per_trial() const;
  // Unnormalised N-point R2C (n/2+1 bins) and C2R, as rocFFT's.
  void forward(const float* d_series, float2* d_spec);
  void inverse(const float2* d_spec, float* d_series);
  // Forward spectrum of the (whitened) series is left in spectrum() until the next call.
  float2* spectrum() const { return fser_.data(); }
  const float* stats() const { return stats_.data(); }  // {mean, rms, std} of the interbin spectrum
  uint64_t n() const { return n_; }
  uint64_t nbins() const { return n_ / 2 + 1; }
  float bin_width() const { return bin_width_; }
  bool uses_fft4() const { return f4_ || mixed_; }  // no rocFFT (power-of-two or mixed-radix four-step passes)
  bool mixed_radix() const { return mixed_; }
  // Allocate whiten_batch's buffers for `count` trials now.
  void reserve_batch(int count);

 private:
  FftPlan& r2c();
  FftPlan& c2r();
  uint64_t n_;
  float tsamp_, bin_width_;
  hipStream_t stream_;
  std::unique_ptr<FftPlan> r2c_, c2r_;  // rocFFT, created on first use
  void ensure_batch(int count);
  void dered_stats(float2* spec, const uint32_t* d_zapmask, float* d_stats, float boundary5, float boundary25);
  bool f4_ = false;
  // n = mm_ * mp_ (mp_ a power of two, mm_ odd): mm_ batched mp_-point
  // complex FFTs on the four-step passes + a length-mm_ combination
  // (kern::mixed_*), so no length needs rocFFT's runtime-compiled kernels
  bool mixed_ = false;
  bool fused_stats_ = true;  // deredden + interbin stats in one pass (PSOUP_WHITEN_FUSED_STATS=0: two kernels)
  uint32_t mm_ = 1;
  uint64_t mp_ = 0;
  kern::Fft4Geom gm_;
  DeviceBuffer<float2> mtab_, mz_, my_, mx_;
  DeviceBuffer<float> mpad_;
  DeviceBuffer<double> maf0_;
  void mixed_fft(const float* src, int gather_mode, void* out, int combine_mode);
  kern::Fft4Geom g4_;
  int bcap_ = 0;  // trials the fft4 batch buffers hold
  DeviceBuffer<float2> tab4_, y4_, x4_, tmp4_;
  DeviceBuffer<float> in4_;
  DeviceBuffer<double> af0_;
  DeviceBuffer<float2> bspec_;
  DeviceBuffer<unsigned long long> bsum_;
  DeviceBuffer<float2> fser_;
  DeviceBuffer<float> m5_, m25_, m125_;
  DeviceBuffer<double> partials_;
  DeviceBuffer<float> stats_;
  DeviceBuffer<unsigned long long> sum_;
};

struct SearchCounters {
  uint64_t dm_trials = 0;
  uint64_t accel_trials = 0;
  uint64_t peaks = 0;
  uint64_t overflows = 0;
  uint64_t harm_in = 0, harm_out = 0;  // candidates into / out of the per-trial harmonic distiller
  uint64_t gpu_distilled = 0, host_distilled = 0;  // trials distilled on the device / on the host
  double whiten_s = 0, accel_s = 0, host_s = 0;
  double accd_s = 0;    // acceleration distillation (host worker time, mostly overlapped)
  double tail_s = 0;    // time collect() waited for the acceleration distillation
};

// The per-DM acceleration distiller a SearchEngine built from p applies
// (pipeline_multi.cu:243: tobs = fft size x tsamp, freq_tol, keep related).
AccelerationDistiller search_accel_distiller(const SearchParams& p);

class SearchEngine {
 public:
  SearchEngine(const SearchParams& p, hipStream_t stream);
  ~SearchEngine();
  // Full Worker::start body for one DM trial (pipeline_multi.cu:147-243):
  // returns the acceleration-distilled candidates of this DM.
  CandidateList search_trial(const uint8_t* d_trial, uint64_t nsamps, float dm, int dm_idx,
                             const std::vector<float>& accs);
  // Batched front end: whiten `count` (<= max_prepare()) trials at d_trials +
  // b*row_stride in one batch, then search each with search_prepared(b, ...).
  // search_trial = prepare(trial, 0, nsamps, 1) + search_prepared(0, ...).
  void prepare(const uint8_t* d_trials, uint64_t row_stride, uint64_t nsamps, int count, int first = 0);
  CandidateList search_prepared(int b, float dm, int dm_idx, const std::vector<float>& accs);
  // Several prepared DMs at once: their acceleration trials are concatenated
  // and cut into batches of K regardless of DM boundaries (a batch's trials
  // may resample different series), so short trial lists still fill batches
  // and the slot pipeline does not drain between DMs.  Returns one
  // acceleration-distilled list per job, identical to search_prepared's.
  struct Job {
    int b;  // prepared series
    float dm;
    int dm_idx;
    std::vector<float> accs;
    // raw: the job is one slice of the DM's acceleration trials (the trials
    // of one DM split over work units, possibly on several ranks): its list
    // is the per-trial harmonic-distilled candidates in trial order, and the
    // acceleration distillation runs once the slices are joined in plan order
    // (accel_distill_slices)
    bool raw = false;
  };
  std::vector<CandidateList> search_prepared_many(const std::vector<Job>& jobs);
  // The same in two halves: search_prepared_many_async returns once every
  // batch has retired and its peaks are on the host, while the per-DM
  // acceleration distillation may still run on the engine's workers; the
  // caller issues its next GPU work (the next DM block) and then collects.
  // Any number of searches may be pending; collect() waits for one and
  // returns its per-job lists (rethrowing a worker's error).
  struct Pending {
    std::vector<CandidateList> out, by_job;
    std::vector<double> accd_t;
    std::mutex mu;
    std::condition_variable cv;
    int remaining = 0;   // acceleration distillation tasks not yet finished
    std::exception_ptr err;
    double accel_s = 0;  // host wall time of the launch and the finish
    // launch / finish state
    std::vector<Job> jobs;
    std::vector<int> job_end;  // flat index one past each job's last trial
    int jobs_sent = 0, next = 0, kc = 0, ntr = 0;
    std::deque<int> inflight;  // slots with a batch in flight
    bool open = false;         // launched, not yet finished
    Stopwatch sw;
    double launch_s = 0;
  };
  std::shared_ptr<Pending> search_prepared_many_async(const std::vector<Job>& jobs);
  // search_prepared_many_async in two halves: search_launch returns once the
  // first (up to two) batches are issued; the caller may then issue other GPU
  // work on the engine's stream (the next DM block's whitening, into the other
  // half of the prepared slots: prepare(..., first)) before search_finish
  // waits for the batches, issues the rest and processes every peak.  One
  // launch at a time (search_finish before the next launch).
  std::shared_ptr<Pending> search_launch(const std::vector<Job>& jobs);
  void search_finish(const std::shared_ptr<Pending>& p);
  std::vector<CandidateList> collect(const std::shared_ptr<Pending>& p);
  int max_prepare() const { return max_prep_; }
  // Allocate up front what prepare(count) and search_prepared_many over
  // `trials` trials would grow on first use (a growth mid-search frees the
  // old buffer: hipFree waits for the whole device, every engine's stream)
  // two: room for a second half of prepared slots [max_prepare, 2 max_prepare)
  // (prepare(..., first = max_prepare) while the first half is searched)
  void reserve(int count, int trials, bool two = false);
  // the acceleration batch search_prepared_many uses for a flat list of ntr trials
  int batch_for(int ntr) const;
  const SearchParams& params() const { return p_; }
  const SearchCounters& counters() const { return ctr_; }
  void reset_counters() { ctr_ = SearchCounters(); }
  int batch_size() const { return K_; }
  int last_batch() const { return last_kc_; }  // batch size of the last search_prepared_many call
  int sub_batch() const { return sub_; }
  int fft_mode() const { return mode_; }
  bool rows_ext() const { return rows_ext_; }  // fft_mode 2 with rocFFT rows (fft4_geometry_rows)
  hipStream_t stream() const { return stream_; }
  float tobs() const { return tobs_; }
  // Debug access to the whitened series / interbin stats of the last searched trial.
  const float* whitened() const { return cur_tim_; }
  // The current search's whitened series (n floats) into dst, from the
  // padded input when prepare() wrote only that (blocking copy).
  void copy_whitened(float* dst) const;
  const float* trial_stats() const { return cur_stats_; }
  const Whitener& whitener() const { return *wh_; }

 private:
  struct Slot {
    DeviceBuffer<kern::PeakRecord> d_peaks;
    // [0] threshold crossings, [1] cluster peaks, [2] distilled candidates;
    // with record regions their counters from [kPeakRegionStride] (rcount)
    DeviceBuffer<uint32_t> d_count;
    PinnedBuffer<kern::PeakRecord> h_peaks;
    PinnedBuffer<uint32_t> h_count;
    // GPU clustering (kern::peak_cluster_batch): segment work/table, the
    // crossings grouped by segment, the cluster peaks; host copies
    DeviceBuffer<uint32_t> d_work;
    DeviceBuffer<uint2> d_sorted, d_clust, d_segtab;
    PinnedBuffer<uint2> h_clust, h_raw, h_segtab;
    // GPU harmonic distillation (kern::harm_distill_batch): distilled
    // candidates and the per-trial table; host copies
    DeviceBuffer<uint2> d_hout, d_ttab;
    PinnedBuffer<uint2> h_hout, h_ttab;
    std::unique_ptr<Event> done, copied;
    int first = 0, count = 0;
  };
  uint32_t* rcount(Slot& s) { return s.d_count.data() + (rlog2_ ? kern::kPeakRegionStride : 0); }
  void ensure_batch_buffers(int k);
  FftPlan& batch_plan(int count);
  void launch_batch(Slot& s, int first, int count);
  void grow_capacity(uint32_t need);
  // first/count/npeaks are the batch's values captured before the slot was
  // re-issued (launch_batch overwrites Slot::first/count/h_count)
  void process_slot(Slot& s, int first, int count, uint32_t npeaks, std::vector<CandidateList>& out_by_job);
  // GPU-clustered batch: segtab is the batch's segment table (snapshot taken
  // before the slot was re-issued), cluster peaks in s.h_clust, raw segments
  // in s.h_raw
  // ttab (GPU harmonic distillation, else null): the batch's per-trial table;
  // distilled trials' candidates in s.h_hout, the host-flagged trials'
  // cluster peaks copied into s.h_clust / s.h_raw at their device offsets
  void process_clustered(Slot& s, int first, int count, const std::vector<uint2>& segtab,
                         const std::vector<uint2>* ttab, std::vector<CandidateList>& out_by_job);
  // per-trial candidates from (idx, snr) cluster peaks of each level, then the
  // harmonic distiller; trials [0, count) over the host pool when heavy.
  // distilled(k, list), when given, fills trial k's already distilled list and
  // returns true, or returns false to send the trial through peaks_of.
  void build_trials(int first, int count, size_t work, const std::function<void(int, int, std::vector<int>&,
                    std::vector<float>&)>& peaks_of, std::vector<CandidateList>& out_by_job,
                    const std::function<bool(int, CandidateList&)>* distilled = nullptr);
  std::vector<uint2> segtab_;  // segment table snapshot of the batch being processed
  std::vector<uint2> ttab_;    // its per-trial distillation table
  bool gpu_cluster_ = true;  // env PSOUP_GPU_CLUSTER=0: cluster on the host (reference path)
  int rlog2_ = 0;            // record regions (SearchParams::peak_region_log2; device clustering only)
  bool gpu_distill_ = true;  // env PSOUP_GPU_DISTILL=0: per-trial harmonic distillation on the host
  kern::HarmDistillParams hdp_{};
  // flat trial list of the current search_prepared_many call
  const std::vector<Job>* jobs_ = nullptr;
  std::vector<int> flat_job_;
  std::vector<float> flat_acc_;
  std::vector<uint32_t> flat_src_;
  DeviceBuffer<uint32_t> d_src_;

  SearchParams p_;
  hipStream_t stream_;
  Stream copy_stream_;
  std::vector<std::unique_ptr<Stream>> aux_;  // further compute streams of the sub-batch pipeline
  std::vector<std::unique_ptr<Event>> joins_;
  Event fork_;
  int sub_ = 0;                    // effective sub-batch size (0 = whole batch on stream_)
  uint64_t n_, nb_;
  float bin_width_, tobs_;
  int nlev_;
  int K_;
  int k_small_ = 1;     // auto short-list batch floor
  int last_kc_ = 0;
  int buf_k_ = 0;       // trials the batch buffers hold
  uint32_t cap_;
  kern::HarmParams hp_{};
  std::vector<PeakBounds> bounds_;
  int hi_ = 0;
  std::unique_ptr<Whitener> wh_;
  DeviceBuffer<float> tim_;    // whitened series of the prepared trials [max_prep_][n_]
  DeviceBuffer<float> wstats_; // their interbin stats [max_prep_][4]
  int prepared_ = 0, max_prep_ = 1;
  const float* cur_tim_ = nullptr;  // trial being searched
  const float* cur_pad_ = nullptr;
  bool pad_direct_ = true;   // whiten into the padded input directly (PSOUP_WHITEN_PAD_DIRECT=0: no)
  bool pad_only_ = false;    // the last prepare() wrote the padded input only (tim_ unwritten)
  const float* cur_stats_ = nullptr;
  DeviceBuffer<uint32_t> zapmask_;
  bool zap_ = false;
  int mode_ = 2;        // effective fft_mode
  kern::Fft4Geom f4_;
  uint64_t pst_ = 1;     // floats per trial of P_
  DeviceBuffer<float2> f4_tab_;
  DeviceBuffer<float> f4_in_;  // padded whitened series read by the fused FFT [max_prep_][insize]
  uint64_t xs_ = 0;     // per-trial stride of spec_ (complex)
  DeviceBuffer<float> res_;
  DeviceBuffer<float2> spec_;
  DeviceBuffer<float> P_;
  // screening bytes of P_ (dev::q8) for the screened harmonic sum: written by
  // the tiled r2c kernel (fft_mode 2); harmonic flag 4 turns the screen off
  bool q8_ = false;
  // harmonic flag 8: P_ is not written; the screen's exact sums recompute
  // their bins from spec_ (kern::HarmFromX)
  bool fromx_ = false;
  // harmonic flag 64 (default): pass B forms P_ (blocked) and Q_ itself
  // (kern::fft4_rowpass_spectrum); no spec_ and no r2c pass
  bool fused_ = false;
  const float2* rt_ = nullptr;  // kern::r2c_twiddle_table(n_ / 2)
  uint64_t qst_ = 0;  // bytes per trial of Q_ (>= hi_, multiple of 64)
  DeviceBuffer<uint8_t> Q_;
  DeviceBuffer<double> af_;
  std::vector<double> af_host_;
  std::map<int, std::unique_ptr<FftPlan>> plans_;
  bool open_ = false;   // a search_launch awaits its search_finish
  int slot_next_ = 0;   // the batch slot the next launch issues into first
  void issue_batch(Pending& pd, int slot);
  void send_done(const std::shared_ptr<Pending>& pd, int processed);
  bool rows_ext_ = false;                // f4_ from fft4_geometry_rows: rocFFT over the rows
  std::unique_ptr<FftPlan> rows_plan_;  // (created on the first batch)
  Slot slots_[2];
  SearchCounters ctr_;
  HarmonicDistiller harm_;
  AccelerationDistiller accd_;
  // host scratch
  std::vector<uint32_t> seg_count_, seg_off_;
  std::vector<kern::PeakRecord> sorted_;
  std::unique_ptr<HostPool> pool_;  // null: serial host processing
  // per-DM acceleration distillation as each DM's last batch retires (last
  // member: destroyed first, its workers drain before accd_ goes away)
  std::unique_ptr<TaskQueue> accq_;
};

// Zap mask for an FFT size (birdiezapper.hpp / kernels.cu:1036-1069 semantics).
std::vector<uint32_t> build_zap_mask(const std::vector<float>& freqs, const std::vector<float>& widths,
                                     float bin_width, uint64_t nbins);

// Host part of FoldOptimiser::calculate_sn (folder.hpp:140-183); the
// negative modulo the reference invokes for bin < nbins/2 is made a proper
// circular index.
void fold_calculate_sn(const float* prof, int bin, int width, int nbins, float* sn1, float* sn2);

struct FoldResult {
  float folded_snr = 0.f;
  double opt_period = 0.0;
  int opt_width = 0;
  int opt_bin = 0;
  std::vector<float> fold;  // [nints][nbins]
  std::vector<float> prof;
};

class FoldEngine {
 public:
  static constexpr int kNbins = 64;
  static constexpr int kNints = 16;
  FoldEngine(uint64_t nsamps, float tsamp, hipStream_t stream);
  // Fold + optimise candidates (period, acc) of one DM trial.
  std::vector<FoldResult> fold_trial(const uint8_t* d_trial, uint64_t trial_nsamps, const std::vector<double>& periods,
                                     const std::vector<float>& accs);
  // Fold + optimise the candidates of ntrials DM trials (trial t at
  // d_trials + t*row_stride, its candidates periods[t], accs[t]): the trials
  // are whitened as batches (one four-step FFT pair per batch), then one
  // accumulate / reduce / optimise launch folds every candidate of a batch
  // and one copy brings the results back (folder.hpp:352-406 per DM).
  std::vector<std::vector<FoldResult>> fold_trials(const uint8_t* d_trials, uint64_t row_stride,
                                                   uint64_t trial_nsamps, int ntrials,
                                                   const std::vector<std::vector<double>>& periods,
                                                   const std::vector<std::vector<float>>& accs);
  // The same for DM trials resident at scattered device rows (the search's
  // kept dedispersed rows): gathered per batch by one copy kernel.
  std::vector<std::vector<FoldResult>> fold_rows(const std::vector<const uint8_t*>& rows, uint64_t trial_nsamps,
                                                 const std::vector<std::vector<double>>& periods,
                                                 const std::vector<std::vector<float>>& accs);
  // Allocate every batch buffer up front (a full batch of trials and
  // njobs_hint candidates), so the fold stage's first batch does not pay it.
  void reserve(int njobs_hint);
  // DM trials whitened per batch (device memory bounds it)
  int max_batch() const { return max_batch_; }
  // Fold + optimise candidates on an already-whitened series (testing).
  std::vector<FoldResult> fold_series(const float* d_series, const std::vector<double>& periods,
                                      const std::vector<float>& accs);
  uint64_t nsamps() const { return n_; }

 private:
  uint64_t n_;
  float tsamp_;
  hipStream_t stream_;
  std::unique_ptr<Whitener> wh_;
  int max_batch_ = 1;
  DeviceBuffer<uint8_t> gathered_;  // fold_rows: one batch of gathered rows
  std::vector<FoldResult> fold_jobs(const float* d_series, const std::vector<kern::FoldJob>& jobs,
                                    const std::vector<double>& periods);
  DeviceBuffer<float> bstats_;
  DeviceBuffer<float> tim_;  // whitened series of the current fold batch [batch][n_]
  DeviceBuffer<float2> shift_table_;
  DeviceBuffer<kern::FoldJob> jobs_;
  DeviceBuffer<float> psum_, folds_, opt_fold_, opt_prof_, opt_val_;
  DeviceBuffer<int32_t> pcount_, opt_int_;
  int chunk_ = 4096;
};

// Multi-beam coincidencer helpers (coincidencer.cpp:124-200): normalise a
// beam (time series and spectrum) and add its indicator (x > thresh) into
// uint8 count arrays.
struct BeamProducts {
  DeviceBuffer<float> series;    // normalised whitened time series [n]
  DeviceBuffer<float> spectrum;  // normalised interbinned spectrum [n/2+1]
};
void coincidencer_beam(const uint8_t* d_trial, uint64_t n, float tsamp, BeamProducts& out, hipStream_t stream);
// Write text outputs (coincidencer.hpp:42-80).
void write_samp_mask(const std::vector<float>& mask, const std::string& filename);
void write_birdie_list(const std::vector<float>& mask, float bin_width, const std::string& filename);

}  // namespace psoup
