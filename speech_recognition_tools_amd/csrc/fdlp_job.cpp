// fdlp_job.cpp -- native JOB runner behind compute-fdlp-feats: the utterance loop of getFeats
// (computeFDLPSpectrogram.py:119-237) for one scp shard, with the host work off the Python
// interpreter:
//   * reader threads read and parse the scp entries ahead of the consumer, in scp order
//     (`<path>`, `<cmd> |` through popen, Kaldi `<ark>:<offset>` wave entries; :125-154);
//   * the consumer applies the reference's per-utterance semantics (skip on read failure, the
//     sr assertion, noise offsets from the numpy-legacy RNG, :135-166), draws the hop jitter
//     (CPython-random replica, :225) and packs device batches into pinned buffers;
//   * each batch is copied in, featurised by fdlp_compute and copied back on one HIP stream, three
//     batch slots in rotation so the copies, the kernels and the host overlap;
//   * a writer thread appends the finished utterances to the Kaldi ark/scp (fdlp_ark_*, written to
//     <name>.tmp and renamed when complete) and the .len lines (:231-237), and the optional global
//     CMVN stats accumulate on the device (fdlp_cmvn_accumulate).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fdlp.h"
#include "fdlp_error.h"

namespace {

using fdlp::fail;

double now_s() {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

// ---- one scp entry ---------------------------------------------------------------------------
struct Utt {
  std::string id;
  bool ok = false;
  bool is_int16 = false;
  int32_t sr = 0, ch = 0;
  int64_t T = 0;
  std::shared_ptr<std::vector<uint8_t>> raw;   // the file bytes; is_int16: the samples point into them
  const int16_t* s16 = nullptr;
  std::shared_ptr<std::vector<double>> f64;    // otherwise (scipy's dtype, converted exactly as numpy does)
  int32_t kind = FDLP_SIG_I16;                  // scipy's dtype of the samples (fdlp_wav_kind)
};

// memcpy jobs (utterance samples -> the pinned batch buffer) on a few threads; a job keeps its source
// alive.  The consumer's copies are handed over in groups (kGroup utterances, or fewer at a wait), so
// the hand-off costs one lock and one wake-up per group, not per utterance.  Single producer.
class CopyPool {
 public:
  explicit CopyPool(int n) {
    for (int t = 0; t < n; ++t) th_.emplace_back([this] { run(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void submit(int tag, void* dst, const void* src, size_t n, std::shared_ptr<void> keep) {
    if (!stage_.empty() && stage_.front().tag != tag) push_stage();
    stage_.push_back(Job{tag, dst, src, n, std::move(keep)});
    if (stage_.size() >= kGroup) push_stage();
  }
  void wait(int tag) {
    push_stage();
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [&] { return pending_[tag] == 0; });
  }

 private:
  static constexpr size_t kGroup = 16;
  struct Job {
    int tag;
    void* dst;
    const void* src;
    size_t n;
    std::shared_ptr<void> keep;
  };
  void push_stage() {
    if (stage_.empty()) return;
    const int tag = stage_.front().tag;
    {
      std::lock_guard<std::mutex> g(m_);
      q_.push_back(std::move(stage_));
      ++pending_[tag];
    }
    stage_ = std::vector<Job>();
    cv_.notify_one();
  }
  void run() {
    for (;;) {
      std::vector<Job> grp;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        grp = std::move(q_.front());
        q_.pop_front();
      }
      for (auto& j : grp) {
        memcpy(j.dst, j.src, j.n);
        j.keep.reset();
      }
      {
        std::lock_guard<std::mutex> g(m_);
        --pending_[grp.front().tag];
      }
      done_.notify_all();
    }
  }
  std::mutex m_;
  std::condition_variable cv_, done_;
  std::deque<std::vector<Job>> q_;
  std::vector<Job> stage_;  // the producer's group being filled (no lock: single producer)
  int pending_[8] = {0};
  bool stop_ = false;
  std::vector<std::thread> th_;
};

bool read_file(const std::string& path, int64_t offset, std::vector<uint8_t>& out) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  bool ok = true;
  if (offset > 0) ok = fseeko(f, offset, SEEK_SET) == 0;
  if (ok && offset >= 0 && offset != 0) {  // Kaldi wave archive entry: one RIFF object at the offset
    uint8_t head[8];
    ok = fread(head, 1, 8, f) == 8 && !memcmp(head, "RIFF", 4);
    if (ok) {
      const uint32_t sz = head[4] | head[5] << 8 | head[6] << 16 | (uint32_t)head[7] << 24;
      out.assign(head, head + 8);
      out.resize(8 + (size_t)sz);
      const size_t got = fread(out.data() + 8, 1, sz, f);
      out.resize(8 + got);
    }
  } else if (ok) {
    // one read of the whole file into a buffer of its size (no growth copies); anything past the
    // size fstat saw (a file still growing) is appended in chunks
    struct stat sb;
    const size_t sz = fstat(fileno(f), &sb) == 0 && S_ISREG(sb.st_mode) ? (size_t)sb.st_size : 0;
    out.resize(sz);
    size_t got = sz ? fread(out.data(), 1, sz, f) : 0;
    out.resize(got);
    if (got == sz) {
      uint8_t buf[1 << 16];
      size_t n;
      while ((n = fread(buf, 1, sizeof buf, f)) > 0) out.insert(out.end(), buf, buf + n);
    }
    ok = !ferror(f);
  }
  fclose(f);
  return ok;
}

bool file_exists(const std::string& p) {
  FILE* f = fopen(p.c_str(), "rb");
  if (f) fclose(f);
  return f != nullptr;
}

// bytes of the RIFF object an scp entry designates (io_pipeline.read_rx_bytes)
bool read_rx_bytes(std::string rx, std::vector<uint8_t>& out) {
  while (!rx.empty() && isspace((unsigned char)rx.back())) rx.pop_back();
  size_t b = 0;
  while (b < rx.size() && isspace((unsigned char)rx[b])) ++b;
  rx = rx.substr(b);
  if (rx.empty()) return false;
  if (rx.back() == '|') {  // subprocess.run(cmd, shell=True, stdout=PIPE) (:131-133)
    FILE* p = popen(rx.substr(0, rx.size() - 1).c_str(), "r");
    if (!p) return false;
    out.clear();
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, p)) > 0) out.insert(out.end(), buf, buf + n);
    pclose(p);  // the reference ignores the command's exit status too
    return true;
  }
  const size_t colon = rx.find_last_of(':');
  if (colon != std::string::npos && colon + 1 < rx.size() &&
      rx.find_first_not_of("0123456789", colon + 1) == std::string::npos && !file_exists(rx) &&
      file_exists(rx.substr(0, colon)))
    return read_file(rx.substr(0, colon), strtoll(rx.c_str() + colon + 1, nullptr, 10), out);
  return read_file(rx, 0, out);
}

void read_entry(const std::string& line, Utt& u) {
  // tokens = line.strip().split(); uttid, inwav = tokens[0], ' '.join(tokens[1:])   (:126-127)
  std::vector<std::string> tok;
  size_t i = 0;
  while (i < line.size()) {
    while (i < line.size() && isspace((unsigned char)line[i])) ++i;
    size_t j = i;
    while (j < line.size() && !isspace((unsigned char)line[j])) ++j;
    if (j > i) tok.push_back(line.substr(i, j - i));
    i = j;
  }
  u.id = tok.empty() ? std::string() : tok[0];
  std::string rx;
  for (size_t k = 1; k < tok.size(); ++k) rx += (k > 1 ? " " : "") + tok[k];
  auto bytes = std::make_shared<std::vector<uint8_t>>();
  if (tok.size() < 2 || !read_rx_bytes(rx, *bytes)) return;
  int32_t sr = 0, ch = 0, i16 = 0;
  int64_t n = 0;
  if (fdlp_wav_decode(bytes->data(), (int64_t)bytes->size(), &sr, &ch, &i16, &n, nullptr) != FDLP_OK) return;
  u.sr = sr;
  u.ch = ch;
  u.T = n;
  u.is_int16 = i16 != 0;
  if (i16 == 2) {  // big-endian (RIFX) 16-bit PCM: scipy returns '>i2', so it is int16 input; swapped copy
    auto swapped = std::make_shared<std::vector<uint8_t>>((size_t)n * ch * 2);
    std::vector<double> v((size_t)n * ch);
    if (fdlp_wav_decode(bytes->data(), (int64_t)bytes->size(), nullptr, nullptr, nullptr, nullptr, v.data()) != FDLP_OK)
      return;
    int16_t* d = (int16_t*)swapped->data();
    for (size_t q = 0; q < v.size(); ++q) d[q] = (int16_t)v[q];
    u.s16 = d;
    u.raw = std::move(swapped);
  } else if (u.is_int16) {  // the samples stay in the file bytes (no copy until the batch buffer)
    int32_t s2, c2;
    int64_t n2;
    const int16_t* smp = nullptr;
    if (fdlp_wav_parse(bytes->data(), (int64_t)bytes->size(), &s2, &c2, &smp, &n2) != FDLP_OK) return;
    u.s16 = smp;
    u.raw = std::move(bytes);
  } else {
    u.f64 = std::make_shared<std::vector<double>>((size_t)n * ch);
    if (fdlp_wav_decode(bytes->data(), (int64_t)bytes->size(), nullptr, nullptr, nullptr, nullptr, u.f64->data()) !=
            FDLP_OK ||
        fdlp_wav_kind(bytes->data(), (int64_t)bytes->size(), &u.kind) != FDLP_OK)
      return;
  }
  u.ok = true;
}

// ---- ordered read-ahead pool -------------------------------------------------------------------
// Readers run up to `depth` entries and about kAheadBytes of file data ahead of the consumer (at least
// one entry, however large).  Wake-ups are targeted: a reader is woken
// only if one is parked on the depth limit, the consumer only when the entry it waits for is in, so
// the per-utterance cost of the hand-off is a lock, not a broadcast to every thread.
class Reader {
 public:
  Reader(std::vector<std::string> lines, int threads, int depth) : lines_(std::move(lines)), depth_(depth) {
    slots_.resize(lines_.size());
    ready_.assign(lines_.size(), 0);
    bytes_.assign(lines_.size(), 0);
    len_.assign(lines_.size(), -1);
    for (int t = 0; t < std::max(1, threads); ++t) th_.emplace_back([this] { run(); });
  }
  ~Reader() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  size_t size() const { return lines_.size(); }
  // waits until every entry is read, or `enough` samples are, or `ms` milliseconds have passed; true (and
  // every entry's sample count, -1 for a failed read, in *lens) if every entry is read
  bool wait_lengths(int64_t enough, int ms, std::vector<int64_t>* lens) {
    std::unique_lock<std::mutex> g(m_);
    ++count_waiters_;
    cv_count_.wait_for(g, std::chrono::milliseconds(ms),
                       [&] { return read_n_ >= lines_.size() || read_samples_ >= enough; });
    --count_waiters_;
    if (read_n_ < lines_.size()) return false;
    *lens = len_;
    return true;
  }
  // entry i (blocks until read); the caller releases it with done(i)
  Utt& get(size_t i) {
    std::unique_lock<std::mutex> g(m_);
    if (!ready_[i]) {
      want_ = i;
      cv_done_.wait(g, [&] { return ready_[i] != 0; });
      want_ = SIZE_MAX;
    }
    return slots_[i];
  }
  void done(size_t i) {
    Utt dead;
    bool wake;
    {
      std::lock_guard<std::mutex> g(m_);
      dead = std::move(slots_[i]);  // freed outside the lock
      ahead_bytes_ -= bytes_[i];
      consumed_ = i + 1;
      wake = parked_ > 0;
    }
    if (wake) cv_.notify_all();
  }

 private:
  void run() {
    auto may_start = [&] {
      return next_ < lines_.size() && next_ < consumed_ + depth_ && (ahead_bytes_ < kAheadBytes || next_ == consumed_);
    };
    for (;;) {
      size_t i;
      {
        std::unique_lock<std::mutex> g(m_);
        if (!(stop_ || may_start())) {
          ++parked_;
          cv_.wait(g, [&] { return stop_ || may_start() || next_ >= lines_.size(); });
          --parked_;
        }
        if (stop_ || next_ >= lines_.size()) return;
        i = next_++;
      }
      Utt u;
      read_entry(lines_[i], u);
      const size_t nb = (u.raw ? u.raw->size() : 0) + (u.f64 ? u.f64->size() * sizeof(double) : 0);
      const bool u_ok = u.ok;
      const int64_t u_T = u.T, smp = u.ok ? u.T * std::max(1, u.ch) : 0;
      bool wake, count;
      {
        std::lock_guard<std::mutex> g(m_);
        slots_[i] = std::move(u);
        bytes_[i] = nb;
        ahead_bytes_ += nb;
        ready_[i] = 1;
        wake = want_ == i;
        ++read_n_;
        read_samples_ += smp;
        len_[i] = u_ok ? u_T : -1;
        count = count_waiters_ > 0;
      }
      if (wake) cv_done_.notify_one();
      if (count) cv_count_.notify_all();
    }
  }
  std::vector<std::string> lines_;
  std::vector<Utt> slots_;
  std::vector<char> ready_;
  size_t next_ = 0, consumed_ = 0, depth_;
  size_t want_ = SIZE_MAX;  // the entry the consumer waits for
  static constexpr size_t kAheadBytes = size_t(256) << 20;
  std::vector<size_t> bytes_;  // file data held by each read entry
  size_t ahead_bytes_ = 0;     // held by entries read and not yet consumed
  int parked_ = 0;          // readers waiting on the depth limit
  bool stop_ = false;
  size_t read_n_ = 0;          // entries read so far
  int64_t read_samples_ = 0;   // their samples
  std::vector<int64_t> len_;   // samples per entry (-1: not read, or the read failed)
  int count_waiters_ = 0;
  std::mutex m_;
  std::condition_variable cv_, cv_done_, cv_count_;
  std::vector<std::thread> th_;
};

// ---- pipeline trace (fdlp_job_opts.trace_path) --------------------------------------------------
struct Trace {
  bool on = false;
  double t0 = 0.0;
  struct Ev {
    double t;
    const char* what;
    int64_t a, b;
  };
  std::mutex m;
  std::vector<Ev> ev;
  void add(const char* what, int64_t a = 0, int64_t b = 0) {
    if (!on) return;
    const double t = now_s() - t0;
    std::lock_guard<std::mutex> g(m);
    ev.push_back({t, what, a, b});
  }
  void dump(const char* path) {
    if (!on || !path) return;
    FILE* f = fopen(path, "w");
    if (!f) return;
    for (const Ev& e : ev)
      fprintf(f, "{\"t\": %.6f, \"ev\": \"%s\", \"a\": %lld, \"b\": %lld}\n", e.t, e.what, (long long)e.a,
              (long long)e.b);
    fclose(f);
  }
};

// ---- part pool: f(0..parts-1) on a few threads and the caller (one caller at a time) --------------
class PartPool {
 public:
  explicit PartPool(int n) {
    for (int t = 0; t < n; ++t) th_.emplace_back([this] { loop(); });
  }
  ~PartPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int threads() const { return (int)th_.size() + 1; }
  void run(int parts, const std::function<void(int)>& f) {
    if (th_.empty() || parts <= 1) {
      for (int i = 0; i < parts; ++i) f(i);
      return;
    }
    {
      std::lock_guard<std::mutex> g(m_);
      f_ = &f;
      parts_ = parts;
      next_ = 0;
      left_ = parts;
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [&] { return left_ == 0; });
    f_ = nullptr;
  }

 private:
  void work() {
    for (;;) {
      const std::function<void(int)>* fn;
      int i;
      {
        std::lock_guard<std::mutex> g(m_);
        if (!f_ || next_ >= parts_) return;
        fn = f_;
        i = next_++;
      }
      (*fn)(i);
      std::lock_guard<std::mutex> g(m_);
      if (--left_ == 0) done_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
    }
  }
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* f_ = nullptr;
  int parts_ = 0, next_ = 0, left_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
  std::vector<std::thread> th_;
};

// ---- batch slots --------------------------------------------------------------------------------
constexpr int kSlots = 3;
constexpr int kMaxPieces = 16;   // D2H pieces per batch (one event each)
constexpr int kRing = 4;         // widened pieces in flight between the widening stage and the writer

struct Slot {
  void* h_pcm = nullptr;       // pinned
  size_t pcm_cap = 0;          // bytes
  void* d_pcm = nullptr;
  size_t d_pcm_cap = 0;
  float* d_out = nullptr;      // the batch's float32 features (the code fallback and the CMVN source)
  size_t out_cap = 0;          // bytes
  int16_t* d_q = nullptr;      // int16 ark codes (codes mode)
  size_t q_cap = 0;            // bytes
  uint32_t* d_qflag = nullptr;
  void* h_dl = nullptr;        // pinned landing buffer of the D2H leg: codes, or float32 features
  size_t dl_cap = 0;           // bytes
  uint32_t* h_qflag = nullptr; // pinned
  hipEvent_t ev_in = nullptr;    // its PCM is on the device
  hipEvent_t ev_comp = nullptr;  // its features are computed
  hipEvent_t ev_piece[kMaxPieces] = {};  // piece j of the D2H leg has landed
  bool busy = false;           // in flight or not yet written
  bool pinned = false;         // h_pcm / h_dl allocated (by the pinning thread)
};

int grow_pinned(void** p, size_t* cap, size_t need) {
  if (*cap >= need) return FDLP_OK;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  const size_t n = std::max(need, *cap * 3 / 2);
  if (hipHostMalloc(p, n, hipHostMallocDefault) != hipSuccess) return fail(FDLP_E_NOMEM, "pinned host allocation failed");
  *cap = n;
  return FDLP_OK;
}

int grow_device(void** p, size_t* cap, size_t need, hipStream_t s) {
  if (*cap >= need) return FDLP_OK;
  if (*p) {
    if (hipStreamSynchronize(s) != hipSuccess) return fail(FDLP_E_HIP, "stream sync failed");
    (void)hipFree(*p);
  }
  *p = nullptr;
  const size_t n = std::max(need, *cap * 3 / 2);
  if (hipMalloc(p, n) != hipSuccess) return fail(FDLP_E_NOMEM, "device allocation failed");
  *cap = n;
  return FDLP_OK;
}

// The samples and output rows of the largest batch each slot will hold, replaying the main loop's
// batching over the job's entries (their sample counts from the reader): batches ramp from
// max(64, max_frames / 32) frames, doubling up to max_frames, hold whole entries, and go round the slots
// in turn.  Frames and rows per entry are the plan's (fdlp_plan.cpp frames_of / out_of, spectrogram mode).
void slot_needs(const std::vector<int64_t>& lens, const fdlp_config& c, size_t nslots, std::vector<size_t>* smp,
                std::vector<size_t>* rows) {
  const double ov = 1.0 - c.overlap_fraction;
  const int64_t hop = std::max(1, (int)((double)c.srate / (1.0 / (ov * c.fduration))));
  const int64_t n = (int64_t)((double)c.srate * c.fduration), d = n % 2 == 0 ? -1 : 0;
  const int64_t cap = std::max(1, c.max_frames);
  int64_t ramp = std::max<int64_t>(64, cap / 32), bf = 0, bs = 0, br = 0;
  size_t j = 0;
  smp->assign(nslots, 0);
  rows->assign(nslots, 0);
  auto put = [&] {
    (*smp)[j % nslots] = std::max((*smp)[j % nslots], (size_t)bs);
    (*rows)[j % nslots] = std::max((*rows)[j % nslots], (size_t)br);
  };
  for (int64_t T : lens) {
    const int64_t F = T + d > 0 ? (T + d - 1) / hop + 1 : 0;
    if (T < 0 || F < 1) continue;
    const int64_t L = (T * (int64_t)c.frate + c.srate - 1) / std::max(1, c.srate);
    if (bf && bf + F > std::min(cap, ramp)) {
      put();
      ++j;
      bf = bs = br = 0;
      ramp = ramp < cap ? 2 * ramp : ramp;
    }
    bf += F;
    bs += T;
    br += L;
  }
  if (bf) put();
}

void free_slot(Slot& sl) {
  if (sl.h_pcm) (void)hipHostFree(sl.h_pcm);
  if (sl.h_dl) (void)hipHostFree(sl.h_dl);
  if (sl.h_qflag) (void)hipHostFree(sl.h_qflag);
  if (sl.d_pcm) (void)hipFree(sl.d_pcm);
  if (sl.d_out) (void)hipFree(sl.d_out);
  if (sl.d_q) (void)hipFree(sl.d_q);
  if (sl.d_qflag) (void)hipFree(sl.d_qflag);
  if (sl.ev_in) (void)hipEventDestroy(sl.ev_in);
  if (sl.ev_comp) (void)hipEventDestroy(sl.ev_comp);
  for (auto& e : sl.ev_piece)
    if (e) (void)hipEventDestroy(e);
  sl = Slot();
}

// ---- what a keep_warm call leaves for the next one -------------------------------------------------
// The plan, the streams and the slots (pinned and device buffers, events) of a JOB, keyed by the
// config bytes (lifter values compared separately), the device and the batch size.
struct Warm {
  fdlp_config key{};
  std::vector<double> lifter;
  int device = -1;
  fdlp_plan* plan = nullptr;
  hipStream_t s = nullptr, s_in = nullptr, s_out = nullptr;
  std::vector<Slot> slots;
  std::vector<std::vector<float>> ring;  // the widening stage's buffers (already faulted in)
};
std::mutex g_warm_m;
Warm* g_warm = nullptr;

fdlp_config warm_key(const fdlp_config& c) {
  fdlp_config k;
  memcpy(&k, &c, sizeof k);
  k.lifter = nullptr;
  return k;
}

void free_warm(Warm* w) {
  if (!w) return;
  int prev = -1;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(w->device);
  for (hipStream_t x : {w->s, w->s_in, w->s_out})
    if (x) (void)hipStreamSynchronize(x);
  for (auto& sl : w->slots) free_slot(sl);
  for (hipStream_t x : {w->s, w->s_in, w->s_out})
    if (x) (void)hipStreamDestroy(x);
  fdlp_plan_destroy(w->plan);
  if (prev >= 0) (void)hipSetDevice(prev);
  delete w;
}

// the parked state if it matches (key, lifter values, device); a parked state that does not is freed
Warm* take_warm(const fdlp_config& c, int device) {
  Warm* w;
  {
    std::lock_guard<std::mutex> g(g_warm_m);
    w = g_warm;
    g_warm = nullptr;
  }
  if (!w) return nullptr;
  const fdlp_config k = warm_key(c);
  bool same = w->device == device && memcmp(&k, &w->key, sizeof k) == 0 && (c.lifter != nullptr) == !w->lifter.empty();
  if (same && c.lifter) same = memcmp(c.lifter, w->lifter.data(), sizeof(double) * (size_t)c.coeff_num) == 0;
  if (same) return w;
  free_warm(w);
  return nullptr;
}

// utterance boundaries of the D2H pieces of a batch: whole utterances, about chunk_rows rows each, at
// most kMaxPieces pieces
std::vector<int32_t> piece_bounds(const std::vector<int64_t>& rows /* n + 1 offsets */, int64_t chunk_rows) {
  const int32_t n = (int32_t)rows.size() - 1;
  const int64_t total = rows.back();
  const int64_t target = std::max<int64_t>(chunk_rows, (total + kMaxPieces - 1) / kMaxPieces);
  std::vector<int32_t> cb{0};
  int64_t start = 0;
  for (int32_t i = 1; i < n; ++i)
    if (rows[i] - start >= target && (int)cb.size() < kMaxPieces) {
      cb.push_back(i);
      start = rows[i];
    }
  cb.push_back(n);
  return cb;
}

// one finished batch on its way to the ark
struct Done {
  int slot = 0;
  int64_t batch = 0;
  std::vector<std::string> ids;
  std::vector<int64_t> rows;   // n + 1 row offsets into the batch's features
  std::vector<int32_t> cb;     // piece boundaries (utterance indices), pieces = cb.size() - 1
  bool codes = false;
  bool mapped = false;
  bool fallback = false;       // codes overflowed: the float32 features were copied instead, into fb
  std::vector<float> fb;
};

struct Piece {
  std::shared_ptr<Done> d;
  int j = 0;
  const float* data = nullptr;  // rows of piece j (nullptr: skip, an error is pending)
  int ring = -1;
};

struct JobState {
  std::mutex m;
  std::condition_variable cv;        // consumer <-> stages, slot releases, pinning
  std::deque<std::shared_ptr<Done>> queue;   // consumer -> widening stage
  std::deque<Piece> pieces;          // widening stage -> writer
  bool finish_a = false, finish_b = false;
  bool ring_busy[kRing] = {false, false, false, false};
  int err = FDLP_OK;
  std::string err_msg;
  int pin_err = FDLP_OK;             // pinning thread failure
  std::string pin_msg;
  void set_err(int e, const std::string& msg) {  // caller holds m
    if (err == FDLP_OK) {
      err = e;
      err_msg = msg;
    }
  }
};

}  // namespace

extern "C" int fdlp_job_release(void) {
  Warm* w;
  {
    std::lock_guard<std::mutex> g(g_warm_m);
    w = g_warm;
    g_warm = nullptr;
  }
  free_warm(w);
  return FDLP_OK;
}

extern "C" int fdlp_job_run(const fdlp_config* cfg, int device, const char* scp_path, const char* outfile,
                            const fdlp_job_opts* o, fdlp_job_stats* st) {
  if (!cfg || !scp_path || !outfile || !o) return fail(FDLP_E_INVALID, "fdlp_job_run: null argument");
  if (o->scp_type != 0 && o->scp_type != 1) return fail(FDLP_E_INVALID, "Invalid type of scp type, it should be either wav or segment");
  if (cfg->mode != FDLP_MODE_SPECTROGRAM) return fail(FDLP_E_INVALID, "fdlp_job_run: spectrogram plans only");
  if (o->noise && o->preprocess == FDLP_PRE_DIFF) return fail(FDLP_E_INVALID, "fdlp_job_run: diff and noise are exclusive");
  if (o->out_codes < -1 || o->out_codes > 1) return fail(FDLP_E_INVALID, "fdlp_job_run: out_codes must be -1, 0 or 1");
  if (o->out_codes == 1 && (o->ark_decimals < 0 || o->out_mapped))
    return fail(FDLP_E_INVALID, "fdlp_job_run: out_codes needs ark_decimals >= 0 and no out_mapped");
  const double t_start = now_s();
  fdlp_job_stats stats{};
  double write_busy = 0.0, widen_busy = 0.0, d2h_wait = 0.0;
  Trace trace;
  trace.on = o->trace_path != nullptr;
  trace.t0 = t_start;
  const bool mapped = o->out_mapped != 0;
  const bool codes = o->out_codes == 1 || (o->out_codes == -1 && !mapped && o->ark_decimals >= 0 && o->ark_decimals <= 3);
  const size_t dl_elem = codes ? sizeof(int16_t) : sizeof(float);
  const int64_t chunk_rows = o->chunk_rows > 0 ? o->chunk_rows : 65536;
  stats.codes = codes ? 1 : 0;

  // scp lines (for line in fid: every line, blank lines included, is an entry of the reference; a
  // blank line raises IndexError there; here blank lines are ignored like the Python drop-in)
  std::vector<std::string> lines;
  {
    FILE* f = fopen(scp_path, "r");
    if (!f) return fail(FDLP_E_IO, std::string("cannot open scp ") + scp_path);
    std::string cur;
    int c;
    while ((c = fgetc(f)) != EOF) {
      if (c == '\n') {
        if (cur.find_first_not_of(" \t\r") != std::string::npos) lines.push_back(cur);
        cur.clear();
      } else {
        cur.push_back((char)c);
      }
    }
    if (cur.find_first_not_of(" \t\r") != std::string::npos) lines.push_back(cur);
    fclose(f);
  }
  stats.n_lines = (int64_t)lines.size();

  constexpr int kReadDepth = 512;  // entries the readers run ahead of the consumer
  Reader reader(lines, std::max(1, o->io_threads), kReadDepth);  // reading starts while the plan is built

  fdlp_config c = *cfg;
  c.max_frames = std::max(1, o->batch_frames);
  // pinned slot sizes for a full int16 batch: the plan's hop (features.py:135, :104, :174) and rows per frame
  const double ov = 1.0 - c.overlap_fraction;
  const int hop0 = (int)((double)c.srate / (1.0 / (ov * c.fduration)));
  const size_t pin_smp = (size_t)c.max_frames * (size_t)(std::max(hop0, 1) + 1);
  const size_t pin_rows = (size_t)c.max_frames * (size_t)((int64_t)hop0 * c.frate / std::max(1, c.srate) + 2);

  Warm* warm = take_warm(c, device);
  stats.warm = warm ? 1 : 0;
  std::vector<Slot> slots = warm ? std::move(warm->slots) : std::vector<Slot>(kSlots);
  std::vector<std::vector<float>> ring = warm && warm->ring.size() == kRing ? std::move(warm->ring)
                                                                         : std::vector<std::vector<float>>(kRing);
  for (auto& sl : slots) sl.pinned = false;  // usable once the pinning thread has checked (or grown) its buffers
  JobState js;
  // slot sizes: a full int16 batch, or -- for a cold call whose scp the readers finish within 10 ms
  // (a job smaller than a batch or so) -- what its batches need: pinning and unpinning cost about 0.1 s
  // per GB, a large part of a short job's process
  std::vector<size_t> slot_smp(slots.size(), pin_smp), slot_rows(slots.size(), pin_rows);
  bool sized = false;
  const bool cold = !warm;
  // pinning thread: page-locking the slots' host buffers overlaps the plan creation and the first reads;
  // slot k becomes usable when slots[k].pinned is set (slots of a warm call are pinned already)
  std::thread pinner([&] {
    std::vector<size_t> want_smp(slots.size(), pin_smp), want_rows(slots.size(), pin_rows);
    std::vector<int64_t> lens;
    // (a job that has read a full batch of samples already gets full-size slots: no wait beyond that; a
    // scp of more than the readers' depth is taken as large without waiting, so its pinning starts at once:
    // the readers park at that depth until the consumer, which waits for `sized`, takes entries)
    constexpr size_t kSizeLines = kReadDepth;
    if (cold && reader.size() <= kSizeLines && reader.wait_lengths((int64_t)pin_smp, 10, &lens)) {
      std::vector<size_t> ns, nr;
      slot_needs(lens, c, slots.size(), &ns, &nr);
      for (size_t k = 0; k < slots.size(); ++k) {
        want_smp[k] = std::min(pin_smp, ns[k] + ns[k] / 16 + 4096);
        want_rows[k] = std::min(pin_rows, nr[k] + nr[k] / 16 + 64);
      }
    }
    {
      std::lock_guard<std::mutex> g(js.m);
      slot_smp = want_smp;
      slot_rows = want_rows;
      sized = true;
    }
    js.cv.notify_all();
    trace.add("sized");
    for (size_t k = 0; k < slots.size(); ++k) {
      const double t0 = now_s();
      void* hp = slots[k].h_pcm;
      size_t pcap = slots[k].pcm_cap;
      void* hd = slots[k].h_dl;
      size_t dcap = slots[k].dl_cap;
      uint32_t* hf = slots[k].h_qflag;
      int e = grow_pinned(&hp, &pcap, want_smp[k] * sizeof(int16_t));
      if (e == FDLP_OK) e = grow_pinned(&hd, &dcap, want_rows[k] * (size_t)std::max(1, c.nfilters) * dl_elem);
      if (e == FDLP_OK && !hf && hipHostMalloc((void**)&hf, 64, hipHostMallocDefault) != hipSuccess)
        e = fail(FDLP_E_NOMEM, "pinned host allocation failed");
      std::lock_guard<std::mutex> g(js.m);
      if (k == 0) stats.pinned_seconds = now_s() - t0;
      slots[k].h_pcm = hp;
      slots[k].pcm_cap = pcap;
      slots[k].h_dl = hd;
      slots[k].dl_cap = dcap;
      slots[k].h_qflag = hf;
      if (e != FDLP_OK) {
        js.pin_err = e;
        js.pin_msg = fdlp::last_error_slot();
        js.cv.notify_all();
        return;
      }
      slots[k].pinned = true;
      js.cv.notify_all();
    }
  });
  auto join_pinner = [&] {
    if (pinner.joinable()) pinner.join();
  };
  fdlp_plan* plan = warm ? warm->plan : nullptr;
  hipStream_t s = warm ? warm->s : nullptr, s_in = warm ? warm->s_in : nullptr,
              s_out = warm ? warm->s_out : nullptr;  // compute, copy-in, copy-out
  const fdlp_config key = warm_key(c);
  std::vector<double> key_lifter;
  if (c.lifter) key_lifter.assign(c.lifter, c.lifter + c.coeff_num);
  delete warm;
  warm = nullptr;
  // a cold call creates its streams on a helper thread while the plan is built, and moves a few MB each way
  // on them once: the first large copy of a stream sets up its DMA queue (~7-8 ms), off the first batches' path
  hipError_t stream_err = hipSuccess;
  std::thread streamer;
  if (cold)
    streamer = std::thread([&] {
      stream_err = hipSetDevice(device);
      for (hipStream_t* x : {&s, &s_in, &s_out})
        if (!*x && stream_err == hipSuccess) stream_err = hipStreamCreateWithFlags(x, hipStreamNonBlocking);
      if (stream_err != hipSuccess) return;
      constexpr size_t kWarmBytes = size_t(4) << 20;
      void *hb = nullptr, *db = nullptr;
      if (hipHostMalloc(&hb, kWarmBytes, hipHostMallocDefault) == hipSuccess && hipMalloc(&db, kWarmBytes) == hipSuccess) {
        for (hipStream_t x : {s_in, s}) {
          (void)hipMemcpyAsync(db, hb, kWarmBytes, hipMemcpyHostToDevice, x);
          (void)hipStreamSynchronize(x);
        }
        (void)hipMemcpyAsync(hb, db, kWarmBytes, hipMemcpyDeviceToHost, s_out);
        (void)hipStreamSynchronize(s_out);
      }
      if (db) (void)hipFree(db);
      if (hb) (void)hipHostFree(hb);
      trace.add("streams_warm");
    });
  const double t_plan = now_s();
  int rc = plan ? FDLP_OK : fdlp_plan_create(&c, device, &plan);
  stats.plan_seconds = now_s() - t_plan;
  if (streamer.joinable()) streamer.join();
  trace.add("plan");
  if (rc == FDLP_OK && stream_err != hipSuccess)
    rc = fail(FDLP_E_HIP, std::string("stream setup: ") + hipGetErrorString(stream_err));
  if (rc != FDLP_OK) {
    join_pinner();
    for (auto& sl : slots) free_slot(sl);
    for (hipStream_t x : {s, s_in, s_out})
      if (x) (void)hipStreamDestroy(x);
    return rc;
  }
  int32_t B = 0;
  fdlp_plan_out_dim(plan, &B);

  int prev_dev = -1;
  (void)hipGetDevice(&prev_dev);
  fdlp_pyrandom* jrng = nullptr;
  fdlp_nprandom* nrng = nullptr;
  fdlp_ark_writer* ark = nullptr;
  int16_t* d_noise = nullptr;
  double* d_cmvn = nullptr;
  hipStream_t s_fb = nullptr;  // the float32 copy of a batch whose codes overflowed
  CopyPool copies(4);  // before cleanup(): drained there before the pinned buffers are freed
  PartPool widen_pool(codes ? 5 : 0);
  std::string len_text;
  std::thread stage_a, stage_b;
  int32_t sr_seen = -1;  // 'sr' of the last successful read (:139; NameError before the first one)

  auto cleanup = [&](int code) -> int {
    std::string keep = code != FDLP_OK ? fdlp::last_error_slot() : std::string();
    trace.add("cleanup");
    join_pinner();
    {
      std::lock_guard<std::mutex> g(js.m);
      js.finish_a = true;
    }
    js.cv.notify_all();
    if (stage_a.joinable()) stage_a.join();
    {
      std::lock_guard<std::mutex> g(js.m);
      js.finish_b = true;
    }
    js.cv.notify_all();
    if (stage_b.joinable()) stage_b.join();
    for (hipStream_t x : {s, s_in, s_out, s_fb})
      if (x) (void)hipStreamSynchronize(x);
    for (int k = 0; k < (int)slots.size(); ++k) copies.wait(k);
    trace.add("joined");
    if (d_noise) (void)hipFree(d_noise);
    if (d_cmvn) (void)hipFree(d_cmvn);
    if (s_fb) (void)hipStreamDestroy(s_fb);
    if (jrng) fdlp_pyrandom_destroy(jrng);
    if (nrng) fdlp_nprandom_destroy(nrng);
    if (ark && code != FDLP_OK) {
      fdlp_ark_abort(ark);  // a failed JOB publishes no partial ark/scp
    } else if (ark) {
      const int rc2 = fdlp_ark_close(ark);
      if (rc2 != FDLP_OK) {
        code = rc2;
        keep = fdlp::last_error_slot();
      }
    }
    trace.add("closed");
    bool parked = false;
    // park for the next call -- only a plan of the key's batch size: a long utterance that rebuilt the plan
    // (c.max_frames = F) would otherwise leave its larger plan under the original key
    if (o->keep_warm && code == FDLP_OK && s && s_in && s_out && c.max_frames == key.max_frames) {
      bool all_pinned = true;
      for (auto& sl : slots) all_pinned = all_pinned && sl.pinned && !sl.busy;
      if (all_pinned) {
        Warm* w = new Warm();
        w->key = key;
        w->lifter = key_lifter;
        w->device = device;
        w->plan = plan;
        w->s = s;
        w->s_in = s_in;
        w->s_out = s_out;
        w->slots = std::move(slots);
        w->ring = std::move(ring);
        Warm* old;
        {
          std::lock_guard<std::mutex> g(g_warm_m);
          old = g_warm;
          g_warm = w;
        }
        free_warm(old);
        parked = true;
      }
    }
    if (!parked) {
      for (auto& sl : slots) free_slot(sl);
      trace.add("slots_freed");
      for (hipStream_t x : {s, s_in, s_out})
        if (x) (void)hipStreamDestroy(x);
      fdlp_plan_destroy(plan);
      trace.add("plan_freed");
    }
    if (prev_dev >= 0) (void)hipSetDevice(prev_dev);
    stats.seconds = now_s() - t_start;
    stats.write_seconds = write_busy;
    stats.widen_seconds = widen_busy;
    stats.d2h_wait_seconds = d2h_wait;
    if (st) *st = stats;
    trace.add("end");
    trace.dump(o->trace_path);
    if (code != FDLP_OK) fdlp::last_error_slot() = keep;
    return code;
  };
#define JOB_TRY(expr) do { int rc_ = (expr); if (rc_ != FDLP_OK) return cleanup(rc_); } while (0)
#define JOB_HIP(expr) do { hipError_t e_ = (expr); if (e_ != hipSuccess) return cleanup(fail(FDLP_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_))); } while (0)

  JOB_HIP(hipSetDevice(device));
  if (!s) JOB_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  if (!s_in) JOB_HIP(hipStreamCreateWithFlags(&s_in, hipStreamNonBlocking));
  if (!s_out) JOB_HIP(hipStreamCreateWithFlags(&s_out, hipStreamNonBlocking));
  trace.add("streams");
  for (auto& sl : slots) {
    if (!sl.ev_in) JOB_HIP(hipEventCreateWithFlags(&sl.ev_in, hipEventDisableTiming));
    if (!sl.ev_comp) JOB_HIP(hipEventCreateWithFlags(&sl.ev_comp, hipEventDisableTiming));
    for (auto& e : sl.ev_piece)
      if (!e) JOB_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (codes && !sl.d_qflag) JOB_HIP(hipMalloc((void**)&sl.d_qflag, 64));
  }
  trace.add("events");
  JOB_TRY(fdlp_pyrandom_create(o->jitter_key, o->jitter_key_len, &jrng));
  if (o->noise) {
    JOB_TRY(fdlp_nprandom_create(o->noise_seed, &nrng));
    JOB_HIP(hipMalloc((void**)&d_noise, sizeof(int16_t) * std::max<int64_t>(o->noise_len, 1)));
    JOB_HIP(hipMemcpy(d_noise, o->noise, sizeof(int16_t) * o->noise_len, hipMemcpyHostToDevice));
  }
  if (o->cmvn_path) {
    JOB_HIP(hipMalloc((void**)&d_cmvn, sizeof(double) * 2 * (B + 1)));
    JOB_HIP(hipMemsetAsync(d_cmvn, 0, sizeof(double) * 2 * (B + 1), s));
  }
  if (codes) JOB_HIP(hipStreamCreateWithFlags(&s_fb, hipStreamNonBlocking));
  const std::string out_s(outfile);
  JOB_TRY(fdlp_ark_open((out_s + ".ark").c_str(), (out_s + ".scp").c_str(), &ark));
  trace.add("opened");

  // stage A (landing + widening): waits for each D2H piece, widens codes into a ring buffer on the part
  // pool (or passes the float32 rows through), and hands the piece to the writer in order
  stage_a = std::thread([&] {
    int64_t seq = 0;
    for (;;) {
      std::shared_ptr<Done> d;
      {
        std::unique_lock<std::mutex> g(js.m);
        js.cv.wait(g, [&] { return js.finish_a || !js.queue.empty(); });
        if (js.queue.empty()) return;
        d = js.queue.front();
        js.queue.pop_front();
      }
      Slot& sl = slots[d->slot];
      const int np = (int)d->cb.size() - 1;
      bool bad = false;
      for (int j = 0; j < np; ++j) {
        const double tw = now_s();
        if (!bad && hipEventSynchronize(sl.ev_piece[j]) != hipSuccess) {
          std::lock_guard<std::mutex> g(js.m);
          js.set_err(FDLP_E_HIP, "device batch failed");
          bad = true;
        }
        d2h_wait += now_s() - tw;
        trace.add("landed", d->batch, j);
        const int64_t r0 = d->rows[d->cb[j]], r1 = d->rows[d->cb[j + 1]];
        const size_t nv = (size_t)(r1 - r0) * (size_t)B;
        Piece pc;
        pc.d = d;
        pc.j = j;
        if (!bad && j == 0 && d->codes && *sl.h_qflag) {  // a code overflowed: the batch's float32 features
          const size_t tot = (size_t)d->rows.back() * (size_t)B;
          d->fb.resize(tot);
          if (hipMemcpyAsync(d->fb.data(), sl.d_out, sizeof(float) * tot, hipMemcpyDeviceToHost, s_fb) != hipSuccess ||
              hipStreamSynchronize(s_fb) != hipSuccess) {
            std::lock_guard<std::mutex> g(js.m);
            js.set_err(FDLP_E_HIP, "D2H copy failed");
            bad = true;
          }
          d->fallback = true;
          std::lock_guard<std::mutex> g(js.m);
          ++stats.n_code_fallbacks;
        }
        if (bad) {
          pc.data = nullptr;
        } else if (!d->codes) {
          pc.data = (const float*)sl.h_dl + (size_t)r0 * B;
        } else if (d->fallback) {
          pc.data = d->fb.data() + (size_t)r0 * B;
        } else {
          const int k = (int)(seq++ % kRing);
          {
            std::unique_lock<std::mutex> g(js.m);
            js.cv.wait(g, [&] { return !js.ring_busy[k]; });
            js.ring_busy[k] = true;
          }
          if (ring[k].size() < nv) ring[k].resize(nv);
          const double t0 = now_s();
          const int16_t* q = (const int16_t*)sl.h_dl + (size_t)r0 * B;
          float* out = ring[k].data();
          const int parts = (int)std::max<size_t>(1, std::min<size_t>((size_t)widen_pool.threads(), nv >> 17));
          widen_pool.run(parts, [&](int i) {
            const size_t a = nv * (size_t)i / parts, b = nv * (size_t)(i + 1) / parts;
            fdlp::q_widen_span(q + a, (int64_t)(b - a), o->ark_decimals, out + a);
          });
          widen_busy += now_s() - t0;
          trace.add("widened", d->batch, j);
          pc.data = out;
          pc.ring = k;
        }
        {
          std::lock_guard<std::mutex> g(js.m);
          js.pieces.push_back(std::move(pc));
        }
        js.cv.notify_all();
      }
    }
  });

  // stage B (writer): ark/scp + .len of the pieces, in order; frees the slot after its last piece
  stage_b = std::thread([&] {
    std::vector<fdlp::ArkItem> items;
    for (;;) {
      Piece pc;
      {
        std::unique_lock<std::mutex> g(js.m);
        js.cv.wait(g, [&] { return js.finish_b || !js.pieces.empty(); });
        if (js.pieces.empty()) return;
        pc = std::move(js.pieces.front());
        js.pieces.pop_front();
      }
      Done& d = *pc.d;
      const double tb = now_s();
      int err = FDLP_OK;
      std::string msg;
      if (pc.data) {
        const int32_t u0 = d.cb[pc.j], u1 = d.cb[pc.j + 1];
        const int64_t base = d.rows[u0];
        items.resize((size_t)(u1 - u0));
        for (int32_t i = u0; i < u1; ++i) {
          const int64_t r0 = d.rows[i], r1 = d.rows[i + 1];
          items[i - u0] = {d.ids[i].c_str(), pc.data + (r0 - base) * B, (int32_t)(r1 - r0)};
          if (o->write_len) len_text += d.ids[i] + " " + std::to_string(r1 - r0) + "\n";  // :235-236
        }
        bool skip;
        {
          std::lock_guard<std::mutex> g(js.m);
          skip = js.err != FDLP_OK;
        }
        if (!skip && fdlp::ark_write_batch(ark, items.data(), items.size(), B) != FDLP_OK) {
          err = FDLP_E_IO;
          msg = fdlp::last_error_slot();
        }
      }
      write_busy += now_s() - tb;
      trace.add("written", d.batch, pc.j);
      {
        std::lock_guard<std::mutex> g(js.m);
        if (pc.ring >= 0) js.ring_busy[pc.ring] = false;
        if (pc.j + 2 == (int)d.cb.size()) slots[d.slot].busy = false;
        if (err != FDLP_OK) js.set_err(err, msg);
      }
      js.cv.notify_all();
    }
  });

  const size_t pcm_elem_i16 = sizeof(int16_t), pcm_elem_f64 = sizeof(double);
  struct Pending {
    std::vector<std::string> ids;
    std::vector<int64_t> off, len, noff, rows;
    std::vector<double> alpha;
    std::vector<uint8_t> jit;
    int64_t frames = 0, samples = 0, out_rows = 0;
    int kind = FDLP_PCM_I16;
  } pend;
  int slot_i = 0;
  int64_t n_batch = 0;
  int32_t ramp = std::max(64, c.max_frames / 32);  // frames of the current batch (see the loop)

  // waits until the slot's previous batch is written, then makes it the current one
  auto acquire_slot = [&](int k) -> int {
    const double ta = now_s();
    std::unique_lock<std::mutex> g(js.m);
    js.cv.wait(g, [&] { return (!slots[k].busy && slots[k].pinned) || js.err != FDLP_OK || js.pin_err != FDLP_OK; });
    stats.slot_wait_seconds += now_s() - ta;
    if (js.err != FDLP_OK) return fail(js.err, js.err_msg);
    if (js.pin_err != FDLP_OK) return fail(js.pin_err, js.pin_msg);
    return FDLP_OK;
  };
  JOB_TRY(acquire_slot(slot_i));

  auto flush = [&]() -> int {
    if (pend.ids.empty()) return FDLP_OK;
    Slot& sl = slots[slot_i];
    trace.add("flush", n_batch, pend.frames);
    const size_t elem = pend.kind == FDLP_PCM_I16 ? pcm_elem_i16 : pcm_elem_f64;
    copies.wait(slot_i);  // every utterance of the batch is in the pinned buffer
    trace.add("copies", n_batch);
    const size_t nval = (size_t)pend.out_rows * B;
    int r = grow_device(&sl.d_pcm, &sl.d_pcm_cap, (size_t)pend.samples * elem, s);
    if (r != FDLP_OK) return r;
    // out_mapped: the OLA kernel stores the features straight into the slot's pinned host buffer (mapped
    // into the device address space), no D2H copy; with --cmvn_stats they stay in device memory for the
    // statistics kernel.  Otherwise: device features (+ codes) and a D2H leg in pieces on the copy-out stream
    float* h_out_dev = nullptr;
    if (mapped && !d_cmvn && hipHostGetDevicePointer((void**)&h_out_dev, sl.h_dl, 0) != hipSuccess) h_out_dev = nullptr;
    if (!h_out_dev) {
      r = grow_device((void**)&sl.d_out, &sl.out_cap, sizeof(float) * nval, s);
      if (r == FDLP_OK && codes) r = grow_device((void**)&sl.d_q, &sl.q_cap, sizeof(int16_t) * nval, s);
      if (r != FDLP_OK) return r;
    }
    // copy-in on its own stream so it overlaps the previous batch's kernels
    if (hipMemcpyAsync(sl.d_pcm, sl.h_pcm, (size_t)pend.samples * elem, hipMemcpyHostToDevice, s_in) != hipSuccess ||
        hipEventRecord(sl.ev_in, s_in) != hipSuccess || hipStreamWaitEvent(s, sl.ev_in, 0) != hipSuccess)
      return fail(FDLP_E_HIP, "H2D copy failed");
    trace.add("h2d", n_batch);
    fdlp_batch b{};
    b.n_utt = (int32_t)pend.ids.size();
    b.pcm_kind = pend.kind;
    b.pcm_dev = sl.d_pcm;
    b.pcm_off = pend.off.data();
    b.utt_len = pend.len.data();
    b.jitter = pend.jit.empty() ? nullptr : pend.jit.data();
    b.noise_dev = o->noise ? d_noise : nullptr;
    b.noise_off = o->noise ? pend.noff.data() : nullptr;
    b.noise_alpha = o->noise ? pend.alpha.data() : nullptr;
    b.out_dev = h_out_dev ? h_out_dev : sl.d_out;
    b.out_row = pend.rows.data();
    b.out_f64_dev = nullptr;
    b.ark_decimals = o->ark_decimals;
    b.preprocess = o->preprocess;
    const bool use_codes = codes && !h_out_dev;
    b.out_q_dev = use_codes ? sl.d_q : nullptr;
    b.out_q_flag_dev = use_codes ? sl.d_qflag : nullptr;
    if (use_codes && hipMemsetAsync(sl.d_qflag, 0, sizeof(uint32_t), s) != hipSuccess)  // the caller zeroes it
      return fail(FDLP_E_HIP, "flag reset failed");
    r = fdlp_compute(plan, &b, s);
    if (r != FDLP_OK) return r;
    trace.add("computed", n_batch);
    if (d_cmvn) {
      r = fdlp_cmvn_accumulate(sl.d_out, pend.out_rows, B, d_cmvn, s);
      if (r != FDLP_OK) return r;
    }
    auto d = std::make_shared<Done>();
    d->slot = slot_i;
    d->batch = n_batch;
    d->codes = use_codes;
    d->mapped = h_out_dev != nullptr;
    d->rows = std::move(pend.rows);
    d->rows.push_back(pend.out_rows);
    if (h_out_dev) {  // the features are in h_dl once the compute stream passes this point
      d->cb = {0, (int32_t)pend.ids.size()};
      if (hipEventRecord(sl.ev_piece[0], s) != hipSuccess) return fail(FDLP_E_HIP, "event record failed");
    } else {
      d->cb = piece_bounds(d->rows, chunk_rows);
      if (hipEventRecord(sl.ev_comp, s) != hipSuccess || hipStreamWaitEvent(s_out, sl.ev_comp, 0) != hipSuccess)
        return fail(FDLP_E_HIP, "event record failed");
      if (use_codes && hipMemcpyAsync(sl.h_qflag, sl.d_qflag, sizeof(uint32_t), hipMemcpyDeviceToHost, s_out) != hipSuccess)
        return fail(FDLP_E_HIP, "D2H copy failed");
      const char* src = use_codes ? (const char*)sl.d_q : (const char*)sl.d_out;
      for (size_t j = 0; j + 1 < d->cb.size(); ++j) {  // copy-out on its own stream (overlaps the next batch)
        const size_t r0 = (size_t)d->rows[d->cb[j]], r1 = (size_t)d->rows[d->cb[j + 1]];
        const size_t off = r0 * B * dl_elem, n = (r1 - r0) * B * dl_elem;
        if ((n && hipMemcpyAsync((char*)sl.h_dl + off, src + off, n, hipMemcpyDeviceToHost, s_out) != hipSuccess) ||
            hipEventRecord(sl.ev_piece[j], s_out) != hipSuccess)
          return fail(FDLP_E_HIP, "D2H copy failed");
      }
    }
    trace.add("launched", n_batch, (int64_t)d->cb.size() - 1);
    d->ids = std::move(pend.ids);
    {
      std::lock_guard<std::mutex> g(js.m);
      sl.busy = true;
      js.queue.push_back(std::move(d));
    }
    js.cv.notify_all();
    if (o->progress_name) fflush(stdout);
    pend = Pending();
    ++n_batch;
    ++stats.n_batches;
    slot_i = (slot_i + 1) % (int)slots.size();
    return acquire_slot(slot_i);
  };

  {  // device buffers of the slot sizes (the pinning thread's), allocated up front (growth stays possible);
     // the pinned host buffers come from the pinning thread (acquire_slot waits for them)
    {
      std::unique_lock<std::mutex> g(js.m);
      js.cv.wait(g, [&] { return sized || js.pin_err != FDLP_OK; });
    }
    trace.add("alloc");
    for (size_t k = 0; k < slots.size(); ++k) {
      Slot& sl = slots[k];
      const size_t smp = slot_smp[k], rows = slot_rows[k];
      JOB_TRY(grow_device(&sl.d_pcm, &sl.d_pcm_cap, smp * sizeof(int16_t), s));
      if (!mapped || o->cmvn_path) JOB_TRY(grow_device((void**)&sl.d_out, &sl.out_cap, rows * B * sizeof(float), s));
      if (codes) JOB_TRY(grow_device((void**)&sl.d_q, &sl.q_cap, rows * B * sizeof(int16_t), s));
    }
  }

  stats.setup_seconds = now_s() - t_start;
  trace.add("setup");
  for (size_t i = 0; i < reader.size(); ++i) {
    const double tw = now_s();
    Utt& u = reader.get(i);
    stats.read_wait_seconds += now_s() - tw;
    const bool skip = !u.ok;
    if (!skip) sr_seen = u.sr;
    if (o->scp_type == 0) {
      if (sr_seen < 0) return cleanup(fail(FDLP_E_INVALID, "name 'sr' is not defined"));  // :144 before any read
      if (sr_seen != o->srate) return cleanup(fail(FDLP_E_INVALID, "Input file has different sampling rate."));
    }
    if (skip) {
      ++stats.n_skipped;
      reader.done(i);
      continue;
    }
    if (u.ch != 1) return cleanup(fail(FDLP_E_INVALID, "multi-channel WAV input is not supported (the reference expects mono)"));
    const int64_t T = u.T;
    int32_t F = 0, L = 0;
    fdlp_geometry(plan, T, &F, &L);
    if (F < 1) return cleanup(fail(FDLP_E_INVALID, "invalid number of data points (0) specified"));
    const int kind = u.is_int16 ? FDLP_PCM_I16 : FDLP_PCM_F64;
    int64_t noff = 0;
    double alpha = 0.0;
    if (o->noise) {  // add_noise_to_wav (features.py:24-31), np.random.rand() per utterance (:166)
      double uu = 0.0;
      JOB_TRY(fdlp_nprandom_rand(nrng, 1, &uu));
      if (kind == FDLP_PCM_I16) JOB_TRY(fdlp_noise_params(u.s16, T, o->noise, o->noise_len, o->snr, uu, &noff, &alpha));
      else JOB_TRY(fdlp_noise_params_any(u.f64->data(), T, u.kind, o->noise, o->noise_len, o->snr, uu, &noff, &alpha));
    }
    if (o->progress_name) printf("%s: Computing Features for file: %s\n", o->progress_name, u.id.c_str());  // :185
    // a batch is one PCM kind and at most max_frames frames
    int32_t cap = c.max_frames;
    // batches ramp up (max_frames / 32, at least 64, doubling per batch) so the device starts after the first few
    // reads and the pipeline fill is short; steady state runs at max_frames
    if (!pend.ids.empty() && (pend.frames + F > std::min(cap, ramp) || pend.kind != kind)) {
      JOB_TRY(flush());
      ramp = ramp < cap ? 2 * ramp : ramp;
    }
    if (F > cap) {  // an utterance longer than a batch: a bigger plan (the Python drop-in does the same)
      JOB_HIP(hipStreamSynchronize(s));
      {
        std::unique_lock<std::mutex> g(js.m);
        js.cv.wait(g, [&] {
          if (js.err != FDLP_OK) return true;
          for (auto& sl : slots)
            if (sl.busy) return false;
          return true;
        });
      }
      fdlp_plan_destroy(plan);
      plan = nullptr;
      c.max_frames = F;
      JOB_TRY(fdlp_plan_create(&c, device, &plan));
      cap = F;
    }
    // append to the current slot's pinned PCM
    Slot& sl = slots[slot_i];
    const size_t elem = kind == FDLP_PCM_I16 ? pcm_elem_i16 : pcm_elem_f64;
    const size_t need = (size_t)(pend.samples + T) * elem;
    if (need > sl.pcm_cap) {
      copies.wait(slot_i);  // the pending copies target the old buffer
      std::vector<uint8_t> keep((size_t)pend.samples * elem);
      if (pend.samples) memcpy(keep.data(), sl.h_pcm, keep.size());
      JOB_TRY(grow_pinned(&sl.h_pcm, &sl.pcm_cap, std::max(need, pin_smp * elem)));  // hop-based estimate; grow_pinned grows 3/2
      if (!keep.empty()) memcpy(sl.h_pcm, keep.data(), keep.size());
    }
    if (kind == FDLP_PCM_I16)
      copies.submit(slot_i, (int16_t*)sl.h_pcm + pend.samples, u.s16, sizeof(int16_t) * T, u.raw);
    else
      copies.submit(slot_i, (double*)sl.h_pcm + pend.samples, u.f64->data(), sizeof(double) * T, u.f64);
    // pinned landing buffer for this batch's rows (float32 in mapped mode: the OLA kernel stores into it)
    const size_t rows_need = (size_t)(pend.out_rows + L);
    const size_t land_elem = mapped ? sizeof(float) : dl_elem;
    if (rows_need * B * land_elem > sl.dl_cap) {
      const size_t nb = std::max(rows_need * B * land_elem, (size_t)c.max_frames * 120 * B * land_elem);
      if (sl.h_dl) (void)hipHostFree(sl.h_dl);
      sl.h_dl = nullptr;
      sl.dl_cap = 0;
      JOB_HIP(hipHostMalloc((void**)&sl.h_dl, nb, hipHostMallocDefault));
      sl.dl_cap = nb;
    }
    pend.kind = kind;
    pend.ids.push_back(u.id);
    pend.off.push_back(pend.samples);
    pend.len.push_back(T);
    pend.noff.push_back(noff);
    pend.alpha.push_back(alpha);
    pend.rows.push_back(pend.out_rows);
    const size_t j0 = pend.jit.size();
    pend.jit.resize(j0 + (size_t)(F - 1));
    if (F > 1) JOB_TRY(fdlp_pyrandom_randbits2(jrng, F - 1, pend.jit.data() + j0));  // randrange(2) (:225)
    pend.frames += F;
    pend.samples += T;
    pend.out_rows += L;
    ++stats.n_done;
    stats.n_samples += T;
    stats.n_frames_out += L;
    reader.done(i);
  }
  JOB_TRY(flush());
  trace.add("read_all");
  {  // wait for the writer to finish the last batches
    std::unique_lock<std::mutex> g(js.m);
    js.cv.wait(g, [&] {
      if (js.err != FDLP_OK) return true;
      for (auto& sl : slots)
        if (sl.busy) return false;
      return true;
    });
    if (js.err != FDLP_OK) return cleanup(fail(js.err, js.err_msg));
  }
  trace.add("drained");
  JOB_HIP(hipStreamSynchronize(s));
  if (o->write_len) {  // <outfile>.len (:232-237), written whole then renamed
    const std::string tmp = out_s + ".len.tmp";
    FILE* f = fopen(tmp.c_str(), "w");
    if (!f) return cleanup(fail(FDLP_E_IO, "cannot open " + tmp));
    const bool ok = fwrite(len_text.data(), 1, len_text.size(), f) == len_text.size();
    if (fclose(f) != 0 || !ok || rename(tmp.c_str(), (out_s + ".len").c_str()) != 0) {
      remove(tmp.c_str());
      return cleanup(fail(FDLP_E_IO, "cannot write " + out_s + ".len"));
    }
  }
  if (d_cmvn) {
    std::vector<double> h(2 * (size_t)(B + 1));
    JOB_HIP(hipMemcpy(h.data(), d_cmvn, sizeof(double) * h.size(), hipMemcpyDeviceToHost));
    JOB_TRY(fdlp_kaldi_write_dmatrix(o->cmvn_path, h.data(), 2, B + 1, 1));
  }
#undef JOB_TRY
#undef JOB_HIP
  return cleanup(FDLP_OK);
}
