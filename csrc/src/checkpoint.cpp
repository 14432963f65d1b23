#include "psoup/checkpoint.hpp"

#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <iomanip>
#include <iterator>
#include <sstream>
#include <thread>
#include <vector>

#include "psoup/common.hpp"
#include "psoup/output.hpp"

namespace psoup {

namespace {

constexpr uint32_t kSpillMagic = 0x4B435350u;  // "PSCK"
constexpr uint32_t kSpillVersion = 1;
// Bump kIdentityVersion whenever the per-DM candidate numerics change in a
// way the build id below does not capture; PSOUP_NUMERICS_ID (generated at
// build time from the kernel and engine sources, cmake/numerics_id.cmake)
// changes with every edit of those sources, so spills written by another
// build are never mixed into a resumed run.
constexpr int kIdentityVersion = 2;
#ifndef PSOUP_NUMERICS_ID
#include "psoup_numerics_id.hpp"
#endif

struct SpillHeader {
  uint32_t magic;
  uint32_t version;
  uint64_t key;
  uint64_t payload_bytes;
  uint64_t payload_hash;
};
static_assert(sizeof(SpillHeader) == 32, "spill header layout");

std::string hex64(uint64_t v) {
  std::ostringstream os;
  os << std::hex << std::setw(16) << std::setfill('0') << v;
  return os.str();
}

// Size and sampled-content hash of a file; "absent" when it cannot be opened.
// Sampled fingerprints (large inputs) also carry the inode and the
// modification time in nanoseconds: a file regenerated in place with the
// same size, differing outside the sampled blocks, still changes its key.
std::string file_fingerprint(const std::string& path, bool sample_only) {
  if (path.empty()) return "none";
  std::ifstream in(path, std::ios::binary);
  if (!in) return "absent";
  std::string stamp;
  if (sample_only) {
    struct stat sb {};
    if (::stat(path.c_str(), &sb) == 0) {
      std::ostringstream st;
      st << ", inode " << sb.st_ino << ", mtime " << sb.st_mtim.tv_sec << "." << std::setw(9) << std::setfill('0')
         << sb.st_mtim.tv_nsec;
      stamp = st.str();
    }
  }
  in.seekg(0, std::ios::end);
  const uint64_t size = static_cast<uint64_t>(in.tellg());
  uint64_t h = fnv1a64(&size, sizeof(size));
  std::vector<char> buf;
  if (!sample_only || size <= (1u << 20)) {
    buf.resize(size);
    in.seekg(0);
    in.read(buf.data(), static_cast<std::streamsize>(size));
    h = fnv1a64(buf.data(), static_cast<size_t>(in.gcount()), h);
  } else {
    constexpr uint64_t kBlock = 4096, kSamples = 16;
    buf.resize(kBlock);
    for (uint64_t s = 0; s < kSamples; ++s) {
      const uint64_t off = (size - kBlock) * s / (kSamples - 1);  // first and last block included
      in.seekg(static_cast<std::streamoff>(off));
      in.read(buf.data(), static_cast<std::streamsize>(kBlock));
      h = fnv1a64(buf.data(), static_cast<size_t>(in.gcount()), h);
    }
  }
  std::ostringstream os;
  os << size << " bytes, hash " << hex64(h) << stamp;
  return os.str();
}

std::string canonical_path(const std::string& p) {
  char buf[PATH_MAX];
  if (!p.empty() && ::realpath(p.c_str(), buf)) return buf;
  return p;
}

}  // namespace

uint64_t fnv1a64(const void* data, size_t n, uint64_t h) {
  const auto* b = static_cast<const unsigned char*>(data);
  for (size_t i = 0; i < n; ++i) {
    h ^= b[i];
    h *= 0x100000001b3ull;
  }
  return h;
}

RunIdentity make_run_identity(const CmdLineOptions& a, const SigprocHeader& hdr) {
  std::ostringstream os;
  os << std::setprecision(9);
  const uint64_t fft = a.size == 0 ? prev_power_of_two(static_cast<uint64_t>(hdr.nsamples)) : a.size;
  os << "peasoup-amd checkpoint identity v" << kIdentityVersion << "\n";
  os << "build: " << PSOUP_NUMERICS_ID << "\n";
  os << "input: " << canonical_path(a.infilename) << "\n";
  os << "input_file: " << file_fingerprint(a.infilename, true) << "\n";
  os << "header: tsamp=" << std::setprecision(17) << hdr.tsamp << " fch1=" << hdr.fch1 << " foff=" << hdr.foff
     << " tstart=" << hdr.tstart << std::setprecision(9) << " nchans=" << hdr.nchans << " nbits=" << hdr.nbits
     << " nifs=" << hdr.nifs << " nsamples=" << hdr.nsamples << "\n";
  os << "dm: start=" << a.dm_start << " end=" << a.dm_end << " tol=" << a.dm_tol << " pulse_width=" << a.dm_pulse_width
     << "\n";
  os << "acc: start=" << a.acc_start << " end=" << a.acc_end << " tol=" << a.acc_tol
     << " pulse_width=" << a.acc_pulse_width << " convention=" << a.accel_convention << "\n";
  os << "fft_size: " << fft << " fft_mode=" << a.fft_mode << "\n";
  os << "search: nharmonics=" << a.nharmonics << " min_snr=" << a.min_snr << " min_freq=" << a.min_freq
     << " max_freq=" << a.max_freq << " max_harm=" << a.max_harm << " freq_tol=" << a.freq_tol << "\n";
  os << "whitening: boundary_5=" << (a.use_boundaries ? a.boundary_5_freq : 0.05f)
     << " boundary_25=" << (a.use_boundaries ? a.boundary_25_freq : 0.5f) << "\n";
  os << "killfile: " << canonical_path(a.killfilename) << " " << file_fingerprint(a.killfilename, false) << "\n";
  os << "zapfile: " << canonical_path(a.zapfilename) << " " << file_fingerprint(a.zapfilename, false) << "\n";
  // numerics-affecting runtime switches: kernel flag words set through the
  // API, and the env knobs that select another arithmetic path
  os << "switches: " << numerics_flags();
  for (const char* k : {"PSOUP_WHITEN_ROCFFT"})
    if (const char* v = std::getenv(k)) os << " " << k << "=" << v;
  os << "\n";
  RunIdentity id;
  id.text = os.str();
  id.key = fnv1a64(id.text.data(), id.text.size());
  return id;
}

std::string spill_path(const std::string& dir, int d0, int d1) {
  std::ostringstream os;
  os << dir << "/dm_" << d0 << "_" << d1 << ".psoc";
  return os.str();
}

void prepare_checkpoint_dir(const std::string& dir, const RunIdentity& id) {
  PSOUP_CHECK(make_dirs(dir), "cannot create checkpoint directory " << dir);
  const std::string manifest = dir + "/manifest.txt";
  const std::string line = "key " + hex64(id.key);
  {
    std::ifstream in(manifest);
    std::string first;
    if (in && std::getline(in, first) && first != line)
      log_info("warning: checkpoint directory " + dir +
               " holds spills of a different run (" + first + "); they are ignored and recomputed");
  }
  std::ostringstream tmp;
  tmp << manifest << ".tmp." << ::getpid() << "." << std::hash<std::thread::id>{}(std::this_thread::get_id());
  {
    std::ofstream out(tmp.str(), std::ios::trunc);
    out << line << "\n" << id.text;
    out.flush();
    PSOUP_CHECK(out.good(), "cannot write " << tmp.str());
  }
  if (std::rename(tmp.str().c_str(), manifest.c_str()) != 0) {
    const int e = errno;
    std::remove(tmp.str().c_str());
    PSOUP_THROW("cannot rename " << tmp.str() << " to " << manifest << ": " << std::strerror(e));
  }
}

SpillStatus load_spill(const std::string& path, uint64_t key, CandidateList& out) {
  std::ifstream in(path, std::ios::binary);
  if (!in) return SpillStatus::Missing;
  std::vector<uint8_t> buf((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  if (buf.size() < sizeof(SpillHeader)) return SpillStatus::Corrupt;
  SpillHeader h;
  std::memcpy(&h, buf.data(), sizeof(h));
  if (h.magic != kSpillMagic || h.version != kSpillVersion) return SpillStatus::Corrupt;
  if (h.key != key) return SpillStatus::Mismatch;
  const uint8_t* payload = buf.data() + sizeof(SpillHeader);
  if (h.payload_bytes != buf.size() - sizeof(SpillHeader) || fnv1a64(payload, h.payload_bytes) != h.payload_hash)
    return SpillStatus::Corrupt;
  try {
    CandidateList c = deserialize_candidates(payload, h.payload_bytes);
    for (auto& x : c) out.push_back(std::move(x));
  } catch (const std::exception&) {
    return SpillStatus::Corrupt;
  }
  return SpillStatus::Loaded;
}

void save_spill(const std::string& path, uint64_t key, const CandidateList& cands) {
  const std::vector<uint8_t> payload = serialize_candidates(cands);
  SpillHeader h{kSpillMagic, kSpillVersion, key, payload.size(), fnv1a64(payload.data(), payload.size())};
  std::ostringstream tmp;
  tmp << path << ".tmp." << ::getpid() << "." << std::hash<std::thread::id>{}(std::this_thread::get_id());
  {
    std::ofstream out(tmp.str(), std::ios::binary | std::ios::trunc);
    PSOUP_CHECK(out.good(), "cannot open " << tmp.str() << " for writing");
    out.write(reinterpret_cast<const char*>(&h), sizeof(h));
    out.write(reinterpret_cast<const char*>(payload.data()), static_cast<std::streamsize>(payload.size()));
    out.flush();
    if (!out.good()) {
      out.close();
      std::remove(tmp.str().c_str());
      PSOUP_THROW("write failed for checkpoint spill " << tmp.str());
    }
  }
  if (std::rename(tmp.str().c_str(), path.c_str()) != 0) {
    const int e = errno;
    std::remove(tmp.str().c_str());
    PSOUP_THROW("cannot rename " << tmp.str() << " to " << path << ": " << std::strerror(e));
  }
}

const char* spill_status_name(SpillStatus s) {
  switch (s) {
    case SpillStatus::Missing: return "missing";
    case SpillStatus::Loaded: return "loaded";
    case SpillStatus::Mismatch: return "mismatch";
    case SpillStatus::Corrupt: return "corrupt";
  }
  return "?";
}

}  // namespace psoup
