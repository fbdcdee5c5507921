// fdlp_host.cpp -- host-side pieces of libfdlp_hip.so that need no device:
//   * CPython `random` replica (MT19937 + init_by_array + randrange(2))  -> OLA hop jitter
//     (computeFDLPSpectrogram.py:21,225)
//   * numpy legacy RandomState replica (init_genrand + 53-bit rand())      -> noise offset
//     (features.py:25)
//   * add_noise_to_wav energies with int16-wrapped squares                  (features.py:24-31)
//   * RIFF/WAVE parser with scipy.io.wavfile.read's formats   (replaces scipy's read, :133,:139)
//   * Kaldi binary ark/scp writer, tmp + rename  (replaces dict2Ark + copy-feats, features.py:63-69)
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <fcntl.h>
#include <linux/falloc.h>
#include <sys/uio.h>
#include <unistd.h>

#include <climits>
#include <algorithm>
#include <new>
#include <string>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/fdlp.h"
#include "fdlp_error.h"

namespace {

struct MT19937 {
  uint32_t mt[624];
  int mti = 625;
  void init_genrand(uint32_t s) {
    mt[0] = s;
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    mti = 624;
  }
  void init_by_array(const uint32_t* key, int len) {
    init_genrand(19650218u);
    int i = 1, j = 0;
    for (int k = (624 > len ? 624 : len); k; --k) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
      ++i;
      ++j;
      if (i >= 624) { mt[0] = mt[623]; i = 1; }
      if (j >= len) j = 0;
    }
    for (int k = 623; k; --k) {
      mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
      ++i;
      if (i >= 624) { mt[0] = mt[623]; i = 1; }
    }
    mt[0] = 0x80000000u;
    mti = 624;
  }
  uint32_t next() {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    if (mti >= 624) {
      int kk;
      for (kk = 0; kk < 624 - 397; ++kk) {
        uint32_t y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
      }
      for (; kk < 623; ++kk) {
        uint32_t y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
        mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
      }
      uint32_t y = (mt[623] & 0x80000000u) | (mt[0] & 0x7fffffffu);
      mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 1u];
      mti = 0;
    }
    uint32_t y = mt[mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
};

}  // namespace

struct fdlp_pyrandom { MT19937 mt; };
struct fdlp_nprandom { MT19937 mt; };

extern "C" {

int fdlp_pyrandom_create(const uint32_t* key, int32_t key_len, fdlp_pyrandom** out) {
  if (!out || key_len < 0 || (key_len > 0 && !key)) return fdlp::fail(FDLP_E_INVALID, "fdlp_pyrandom_create: bad args");
  auto* r = new (std::nothrow) fdlp_pyrandom;
  if (!r) return fdlp::fail(FDLP_E_NOMEM, "fdlp_pyrandom_create: out of memory");
  // CPython random.seed(int): key = 32-bit words of |seed|, at least one word ([0] for 0)
  const uint32_t zero = 0;
  if (key_len == 0) r->mt.init_by_array(&zero, 1);
  else r->mt.init_by_array(key, key_len);
  *out = r;
  return FDLP_OK;
}

int fdlp_pyrandom_randbits2(fdlp_pyrandom* rng, int64_t n, uint8_t* out) {
  if (!rng || n < 0 || (n > 0 && !out)) return fdlp::fail(FDLP_E_INVALID, "fdlp_pyrandom_randbits2: bad args");
  // randrange(2) -> _randbelow_with_getrandbits(2): k = 2, r = getrandbits(2) until r < 2
  for (int64_t i = 0; i < n; ++i) {
    uint32_t r;
    do { r = rng->mt.next() >> 30; } while (r >= 2u);
    out[i] = (uint8_t)r;
  }
  return FDLP_OK;
}

int fdlp_pyrandom_destroy(fdlp_pyrandom* rng) {
  delete rng;
  return FDLP_OK;
}

int fdlp_nprandom_create(uint32_t seed, fdlp_nprandom** out) {
  if (!out) return fdlp::fail(FDLP_E_INVALID, "fdlp_nprandom_create: bad args");
  auto* r = new (std::nothrow) fdlp_nprandom;
  if (!r) return fdlp::fail(FDLP_E_NOMEM, "fdlp_nprandom_create: out of memory");
  r->mt.init_genrand(seed);  // numpy legacy seeding of an int seed
  *out = r;
  return FDLP_OK;
}

int fdlp_nprandom_rand(fdlp_nprandom* rng, int64_t n, double* out) {
  if (!rng || n < 0 || (n > 0 && !out)) return fdlp::fail(FDLP_E_INVALID, "fdlp_nprandom_rand: bad args");
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t a = rng->mt.next() >> 5, b = rng->mt.next() >> 6;
    out[i] = (a * 67108864.0 + b) / 9007199254740992.0;
  }
  return FDLP_OK;
}

int fdlp_nprandom_destroy(fdlp_nprandom* rng) {
  delete rng;
  return FDLP_OK;
}

int fdlp_noise_params(const int16_t* sig, int64_t T, const int16_t* noise, int64_t noise_len, double snr,
                      double u, int64_t* off, double* alpha) {
  if (!sig || !noise || !off || !alpha || T <= 0) return fdlp::fail(FDLP_E_INVALID, "fdlp_noise_params: bad args");
  // rand_num = int(floor(rand() * (len(noise) - len(sig))))            (features.py:25)
  const double span = (double)(noise_len - T);
  const int64_t o = (int64_t)floor(u * span);
  if (o < 0 || o + T > noise_len)
    return fdlp::fail(FDLP_E_INVALID, "noise file shorter than the utterance (reference slices a short noise)");
  // E = mean(x**2) with int16 squares (wrapping), accumulated exactly  (features.py:27-28)
  int64_t es = 0, en = 0;
  for (int64_t t = 0; t < T; ++t) {
    es += (int16_t)(uint16_t)((uint32_t)(int32_t)sig[t] * (uint32_t)(int32_t)sig[t]);
    en += (int16_t)(uint16_t)((uint32_t)(int32_t)noise[o + t] * (uint32_t)(int32_t)noise[o + t]);
  }
  const double Es = (double)es / (double)T, En = (double)en / (double)T;
  *alpha = sqrt(Es / (En * pow(10.0, snr / 10.0)));  // (features.py:29)
  *off = o;
  return FDLP_OK;
}

}  // extern "C"

// numpy's float reduction as np.mean runs it (numpy/_core/src/umath/loops_utils.h.src pairwise_sum): the
// array is fed to the add loop in 8192-element chunks (the iterator's buffer), each chunk summed pairwise
// (8 accumulators up to 128 elements, halves above, the halves cut at a multiple of 8) and added to the
// running result, which starts at 0.  Acc is the reduction dtype (float for float32 input, double otherwise);
// pinned against np.mean in tests/test_noise_kinds.py.
template <typename Acc>
static Acc np_pairwise(const Acc* a, int64_t n) {
  if (n < 8) {
    Acc res = 0;
    for (int64_t i = 0; i < n; ++i) res = res + a[i];
    return res;
  }
  if (n <= 128) {
    Acc r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] = r[j] + a[i + j];
    Acc res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res = res + a[i];
    return res;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return np_pairwise(a, n2) + np_pairwise(a + n2, n - n2);
}

// np.mean(sig ** 2) with sig in scipy's dtype `kind` (its values given as doubles): the square in that dtype
// (integers wrap, float32 rounds), then the chunked pairwise sum of np_pairwise in the reduction dtype
static double np_mean_square(const double* sig, int64_t T, int kind) {
  constexpr int64_t kChunk = 8192;
  if (kind == FDLP_SIG_F32) {
    std::vector<float> sq((size_t)std::min(T, kChunk));
    float res = 0.0f;
    for (int64_t c0 = 0; c0 < T; c0 += kChunk) {
      const int64_t n = std::min(kChunk, T - c0);
      for (int64_t i = 0; i < n; ++i) {
        const float x = (float)sig[c0 + i];
        sq[(size_t)i] = x * x;
      }
      res = res + np_pairwise(sq.data(), n);
    }
    return (double)(res / (float)T);  // np.float32 scalar / int count: a float32 division (NEP 50)
  }
  std::vector<double> sq((size_t)std::min(T, kChunk));
  double res = 0.0;
  for (int64_t c0 = 0; c0 < T; c0 += kChunk) {
    const int64_t n = std::min(kChunk, T - c0);
    for (int64_t i = 0; i < n; ++i) {
      const double v = sig[c0 + i];
      double q;
      switch (kind) {
        case FDLP_SIG_U8: { const uint8_t x = (uint8_t)(int)v; q = (double)(uint8_t)(x * x); break; }
        case FDLP_SIG_I16: { const int16_t x = (int16_t)v; q = (double)(int16_t)(uint16_t)((uint32_t)(int32_t)x * (uint32_t)(int32_t)x); break; }
        case FDLP_SIG_I32: { const int32_t x = (int32_t)v; q = (double)(int32_t)((uint32_t)x * (uint32_t)x); break; }
        case FDLP_SIG_I64: { const int64_t x = (int64_t)v; q = (double)(int64_t)((uint64_t)x * (uint64_t)x); break; }
        default: q = v * v; break;  // float64
      }
      sq[(size_t)i] = q;
    }
    res = res + np_pairwise(sq.data(), n);
  }
  return res / (double)T;
}

extern "C" {

int fdlp_noise_params_any(const double* sig, int64_t T, int32_t kind, const int16_t* noise, int64_t noise_len,
                          double snr, double u, int64_t* off, double* alpha) {
  if (!sig || !noise || !off || !alpha || T <= 0 || kind < FDLP_SIG_U8 || kind > FDLP_SIG_F64)
    return fdlp::fail(FDLP_E_INVALID, "fdlp_noise_params_any: bad args");
  const double span = (double)(noise_len - T);  // features.py:25
  const int64_t o = (int64_t)floor(u * span);
  if (o < 0 || o + T > noise_len)
    return fdlp::fail(FDLP_E_INVALID, "noise file shorter than the utterance (reference slices a short noise)");
  int64_t en = 0;  // the int16 noise's wrapped squares, exactly (features.py:28)
  for (int64_t t = 0; t < T; ++t)
    en += (int16_t)(uint16_t)((uint32_t)(int32_t)noise[o + t] * (uint32_t)(int32_t)noise[o + t]);
  const double Es = np_mean_square(sig, T, kind), En = (double)en / (double)T;
  *alpha = sqrt(Es / (En * pow(10.0, snr / 10.0)));  // (features.py:29)
  *off = o;
  return FDLP_OK;
}

// Compact ark codes -> the float32 ark values (fdlp_batch.out_q_dev, fdlp_device.h q_code): the device
// stores (float)(k / 10^d) in out_dev; here the same two IEEE operations on the same k, so the floats
// are bitwise the ones the device would have written.  -32768 is -0.0.  The 65536 values of a decimals
// setting are computed once into a table (a lookup per code instead of a double division).
static float q_value(int k, double scale10) { return k == -32768 ? -0.0f : (float)((double)k / scale10); }

static const float* q_table(int decimals, double scale10) {
  constexpr int kTables = 10;
  static std::once_flag once[kTables];
  static std::vector<float> tab[kTables];
  if (decimals >= kTables) return nullptr;
  std::call_once(once[decimals], [&] {
    tab[decimals].resize(65536);
    for (int k = -32768; k < 32768; ++k) tab[decimals][k + 32768] = q_value(k, scale10);
  });
  return tab[decimals].data();
}

static void q_widen_range(const int16_t* q, int64_t n, const float* lut, double scale10, float* out) {
  if (lut) {
    for (int64_t i = 0; i < n; ++i) out[i] = lut[(int)q[i] + 32768];
  } else {
    for (int64_t i = 0; i < n; ++i) out[i] = q_value(q[i], scale10);
  }
}

int fdlp_q_widen(const int16_t* q, int64_t n, int32_t decimals, float* out, int32_t threads) {
  if (n < 0 || (n > 0 && (!q || !out)) || decimals < 0) return fdlp::fail(FDLP_E_INVALID, "fdlp_q_widen: bad args");
  double scale10 = 1.0;
  for (int i = 0; i < decimals; ++i) scale10 *= 10.0;  // as launch_ola_log
  const float* lut = n >= 4096 ? q_table(decimals, scale10) : nullptr;
  const int64_t nt = std::max<int64_t>(1, std::min<int64_t>(threads, n / (int64_t(1) << 16)));
  if (nt <= 1) {
    q_widen_range(q, n, lut, scale10, out);
    return FDLP_OK;
  }
  std::vector<std::thread> th;
  for (int64_t t = 1; t < nt; ++t) {
    const int64_t a = n * t / nt, b = n * (t + 1) / nt;
    th.emplace_back(q_widen_range, q + a, b - a, lut, scale10, out + a);
  }
  q_widen_range(q, n / nt, lut, scale10, out);
  for (auto& x : th) x.join();
  return FDLP_OK;
}

// ---------------------------------------------------------------------------------------------
// WAV
// ---------------------------------------------------------------------------------------------
static uint32_t rd32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
static uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }

// The data chunk of a RIFF/RIFX/WAVE buffer and its format, as scipy.io.wavfile.read sees it
// (scipy/io/wavfile.py _read_fmt_chunk / _read_data_chunk): PCM of 1..64 bits (<= 8 bits unsigned,
// 3/5/6/7-byte containers left-justified into int32/int64), IEEE float 32/64, WAVE_FORMAT_EXTENSIBLE.
struct WavInfo {
  int32_t sr = 0, ch = 0;
  int fmt = 0, bits = 0, bps = 0;  // format tag, bits per sample, container bytes per sample
  bool big = false;
  const uint8_t* data = nullptr;
  int64_t frames = 0;  // samples per channel
};

static uint32_t rdu32(const uint8_t* p, bool big) {
  return big ? ((uint32_t)p[0] << 24 | p[1] << 16 | p[2] << 8 | p[3]) : rd32(p);
}
static uint16_t rdu16(const uint8_t* p, bool big) { return big ? (uint16_t)(p[0] << 8 | p[1]) : rd16(p); }

static int wav_info(const uint8_t* buf, int64_t len, WavInfo* w) {
  if (!buf || len < 12 || (memcmp(buf, "RIFF", 4) && memcmp(buf, "RIFX", 4)) || memcmp(buf + 8, "WAVE", 4))
    return fdlp::fail(FDLP_E_IO, "not a RIFF/WAVE buffer");
  w->big = !memcmp(buf, "RIFX", 4);
  int64_t pos = 12;
  int fmt_ok = 0, block_align = 0;
  while (pos + 8 <= len) {
    const uint8_t* h = buf + pos;
    const uint32_t sz = rdu32(h + 4, w->big);
    const int64_t body = pos + 8;
    if (!memcmp(h, "fmt ", 4)) {
      if (sz < 16 || body + 16 > len) return fdlp::fail(FDLP_E_IO, "truncated fmt chunk");
      w->fmt = rdu16(buf + body, w->big);
      w->ch = rdu16(buf + body + 2, w->big);
      w->sr = (int32_t)rdu32(buf + body + 4, w->big);
      block_align = rdu16(buf + body + 12, w->big);
      w->bits = rdu16(buf + body + 14, w->big);
      if (w->fmt == 0xFFFE && sz >= 18) {  // WAVE_FORMAT_EXTENSIBLE: subformat GUID {XXXXXXXX-0000-0010-8000-00AA00389B71}
        if (body + 18 > len || rdu16(buf + body + 16, w->big) < 22 || body + 40 > len)
          return fdlp::fail(FDLP_E_IO, "Binary structure of wave file is not compliant");
        static const uint8_t tail_le[12] = {0, 0, 0x10, 0, 0x80, 0, 0, 0xAA, 0, 0x38, 0x9B, 0x71};
        static const uint8_t tail_be[12] = {0, 0, 0, 0x10, 0x80, 0, 0, 0xAA, 0, 0x38, 0x9B, 0x71};
        if (!memcmp(buf + body + 28, w->big ? tail_be : tail_le, 12)) w->fmt = (int)rdu32(buf + body + 24, w->big);
      }
      fmt_ok = 1;
    } else if (!memcmp(h, "data", 4)) {
      if (!fmt_ok) return fdlp::fail(FDLP_E_IO, "data chunk before fmt chunk");
      if (w->ch == 0) return fdlp::fail(FDLP_E_IO, "zero channels");
      w->bps = block_align / w->ch;
      if (w->bps < 1) return fdlp::fail(FDLP_E_IO, "block align smaller than the channel count");
      if (w->fmt == 1) {
        if (w->bits < 1 || w->bits > 64 || w->bps > 8) return fdlp::fail(FDLP_E_IO, "unsupported PCM bit depth");
      } else if (w->fmt == 3) {
        if ((w->bits != 32 && w->bits != 64) || (w->bps != 4 && w->bps != 8))
          return fdlp::fail(FDLP_E_IO, "unsupported floating-point bit depth");
      } else {
        return fdlp::fail(FDLP_E_IO, "unknown wave format (only PCM and IEEE float are read)");
      }
      const int64_t avail = len - body;
      // scipy reads what is there when the size field is larger (sox pipes write 0xFFFFFFFF)
      int64_t nbytes = (int64_t)sz > avail ? avail : (int64_t)sz;
      if (sz == 0 || sz == 0xFFFFFFFFu) nbytes = avail;
      w->data = buf + body;
      w->frames = nbytes / w->bps / w->ch;
      return FDLP_OK;
    }
    pos = body + sz + (sz & 1);
  }
  return fdlp::fail(FDLP_E_IO, "no data chunk");
}

// sample i (interleaved index) as the value scipy returns, converted to double
static double wav_sample(const WavInfo& w, int64_t i) {
  const uint8_t* p = w.data + i * w.bps;
  if (w.fmt == 3) {
    if (w.bps == 4) {
      uint32_t u = rdu32(p, w.big);
      float f;
      memcpy(&f, &u, 4);
      return (double)f;
    }
    uint64_t u = w.big ? ((uint64_t)rdu32(p, true) << 32 | rdu32(p + 4, true)) : ((uint64_t)rd32(p + 4) << 32 | rd32(p));
    double d;
    memcpy(&d, &u, 8);
    return d;
  }
  if (w.bits <= 8) return (double)p[0];  // unsigned 8-bit (scipy 'u1')
  // signed integer container of bps bytes; 3/5/6/7-byte containers are left-justified into 4/8 bytes
  const int cont = (w.bps == 1 || w.bps == 2 || w.bps == 4 || w.bps == 8) ? w.bps : (w.bps == 3 ? 4 : 8);
  uint64_t u = 0;
  for (int b = 0; b < w.bps; ++b) {
    const uint64_t byte = w.big ? p[b] : p[w.bps - 1 - b];  // most significant first
    u = (u << 8) | byte;
  }
  u <<= 8 * (cont - w.bps);
  const int sh = 64 - 8 * cont;
  return (double)((int64_t)(u << sh) >> sh);
}

int fdlp_wav_parse(const uint8_t* buf, int64_t len, int32_t* srate, int32_t* channels, const int16_t** samples,
                   int64_t* n_samples) {
  WavInfo w;
  int rc = wav_info(buf, len, &w);
  if (rc != FDLP_OK) return rc;
  if (w.fmt != 1 || w.bits != 16 || w.bps != 2 || w.big) return fdlp::fail(FDLP_E_IO, "only PCM16 WAV is supported");
  *srate = w.sr;
  *channels = w.ch;
  *samples = (const int16_t*)w.data;
  *n_samples = w.frames;
  return FDLP_OK;
}

int fdlp_wav_decode(const uint8_t* buf, int64_t len, int32_t* srate, int32_t* channels, int32_t* is_int16,
                    int64_t* n_samples, double* out) {
  WavInfo w;
  int rc = wav_info(buf, len, &w);
  if (rc != FDLP_OK) return rc;
  if (srate) *srate = w.sr;
  if (channels) *channels = w.ch;
  // 16-bit PCM is what scipy returns as int16 (RIFF '<i2' or RIFX '>i2'): 1 = little-endian (the samples
  // can be used in place, fdlp_wav_parse), 2 = big-endian (decode, then the values are int16)
  if (is_int16) *is_int16 = (w.fmt == 1 && w.bits > 8 && w.bps == 2) ? (w.big ? 2 : 1) : 0;
  if (n_samples) *n_samples = w.frames;
  if (out) {
    const int64_t n = w.frames * w.ch;
    for (int64_t i = 0; i < n; ++i) out[i] = wav_sample(w, i);
  }
  return FDLP_OK;
}

int fdlp_wav_kind(const uint8_t* buf, int64_t len, int32_t* kind) {
  if (!kind) return fdlp::fail(FDLP_E_INVALID, "fdlp_wav_kind: bad args");
  WavInfo w;
  int rc = wav_info(buf, len, &w);
  if (rc != FDLP_OK) return rc;
  if (w.fmt == 3) {
    *kind = w.bps == 4 ? FDLP_SIG_F32 : FDLP_SIG_F64;
  } else if (w.bits <= 8) {
    *kind = FDLP_SIG_U8;
  } else {
    const int cont = (w.bps == 1 || w.bps == 2 || w.bps == 4 || w.bps == 8) ? w.bps : (w.bps == 3 ? 4 : 8);
    *kind = cont == 2 ? FDLP_SIG_I16 : (cont == 4 ? FDLP_SIG_I32 : FDLP_SIG_I64);
  }
  return FDLP_OK;
}

// ---------------------------------------------------------------------------------------------
// Kaldi ark/scp writer: "<utt> \0B" + "FM " + <int32 size=4 rows> + <int32 size=4 cols> + data
// ---------------------------------------------------------------------------------------------
struct fdlp_ark_writer {
  FILE* ark = nullptr;
  FILE* scp = nullptr;
  std::string ark_abs;                   // absolute path of the final ark (what the scp lines name)
  std::string ark_path, scp_path;        // final names
  std::string ark_tmp, scp_tmp;          // written here, renamed by fdlp_ark_close
  bool failed = false;
};

// absolute form of a path that may not exist yet: realpath of its directory + the file name
static std::string abs_path(const std::string& p) {
  const size_t slash = p.find_last_of('/');
  const std::string dir = slash == std::string::npos ? "." : (slash == 0 ? "/" : p.substr(0, slash));
  const std::string base = slash == std::string::npos ? p : p.substr(slash + 1);
  char* d = realpath(dir.c_str(), nullptr);
  std::string r = d ? std::string(d) + (std::string(d) == "/" ? "" : "/") + base : p;
  free(d);
  return r;
}

int fdlp_ark_open(const char* ark_path, const char* scp_path, fdlp_ark_writer** out) {
  if (!ark_path || !out) return fdlp::fail(FDLP_E_INVALID, "fdlp_ark_open: bad args");
  auto* w = new (std::nothrow) fdlp_ark_writer;
  if (!w) return fdlp::fail(FDLP_E_NOMEM, "fdlp_ark_open: out of memory");
  w->ark_path = ark_path;
  w->ark_tmp = w->ark_path + ".tmp";
  w->ark = fopen(w->ark_tmp.c_str(), "wb");
  if (!w->ark) {
    delete w;
    return fdlp::fail(FDLP_E_IO, std::string("cannot open ark ") + ark_path);
  }
  if (scp_path) {
    w->scp_path = scp_path;
    w->scp_tmp = w->scp_path + ".tmp";
    w->scp = fopen(w->scp_tmp.c_str(), "w");
    if (!w->scp) {
      fclose(w->ark);
      remove(w->ark_tmp.c_str());
      delete w;
      return fdlp::fail(FDLP_E_IO, std::string("cannot open scp ") + scp_path);
    }
  }
  w->ark_abs = abs_path(w->ark_path);
  *out = w;
  return FDLP_OK;
}

int fdlp_ark_write(fdlp_ark_writer* w, const char* utt, const float* mat, int32_t rows, int32_t cols) {
  if (!w || !utt || rows < 0 || cols < 0 || (rows * (int64_t)cols > 0 && !mat))
    return fdlp::fail(FDLP_E_INVALID, "fdlp_ark_write: bad args");
  if (fprintf(w->ark, "%s ", utt) < 0) return w->failed = true, fdlp::fail(FDLP_E_IO, "ark write failed");
  const long offset = ftell(w->ark);
  const char hdr[] = {'\0', 'B', 'F', 'M', ' '};
  const char four = 4;
  int ok = fwrite(hdr, 1, 5, w->ark) == 5;
  ok &= fwrite(&four, 1, 1, w->ark) == 1;
  ok &= fwrite(&rows, 4, 1, w->ark) == 1;
  ok &= fwrite(&four, 1, 1, w->ark) == 1;
  ok &= fwrite(&cols, 4, 1, w->ark) == 1;
  const size_t n = (size_t)rows * (size_t)cols;
  if (n) ok &= fwrite(mat, sizeof(float), n, w->ark) == n;
  if (!ok) return w->failed = true, fdlp::fail(FDLP_E_IO, "ark write failed");
  if (w->scp && fprintf(w->scp, "%s %s:%ld\n", utt, w->ark_abs.c_str(), offset) < 0)
    return w->failed = true, fdlp::fail(FDLP_E_IO, "scp write failed");
  return FDLP_OK;
}

}  // extern "C" (the batch writer below is internal C++)

namespace fdlp {
void q_widen_span(const int16_t* q, int64_t n, int32_t decimals, float* out) {
  double scale10 = 1.0;
  for (int i = 0; i < decimals; ++i) scale10 *= 10.0;
  q_widen_range(q, n, q_table(decimals, scale10), scale10, out);
}
}  // namespace fdlp


namespace fdlp {
int ark_write_batch(fdlp_ark_writer* w, const ArkItem* items, size_t n, int32_t cols) {
  if (!w || (n && !items) || cols < 0) return fail(FDLP_E_INVALID, "ark_write_batch: bad args");
  if (fflush(w->ark) != 0) return w->failed = true, fail(FDLP_E_IO, "ark write failed");
  const int fd = fileno(w->ark);
  off_t pos = lseek(fd, 0, SEEK_CUR);
  if (pos < 0) return w->failed = true, fail(FDLP_E_IO, "ark seek failed");
  constexpr size_t kChunk = 512;  // utterances per writev (2 iovecs each, <= IOV_MAX)
  std::vector<char> hdr;
  std::vector<size_t> hoff;
  std::vector<struct iovec> iov;
  for (size_t i0 = 0; i0 < n; i0 += kChunk) {
    const size_t i1 = std::min(n, i0 + kChunk);
    hdr.clear();
    hoff.clear();
    for (size_t i = i0; i < i1; ++i) {  // "<utt> \0BFM \4<rows>\4<cols>"
      const ArkItem& it = items[i];
      if (!it.id || it.rows < 0 || ((int64_t)it.rows * cols > 0 && !it.data))
        return w->failed = true, fail(FDLP_E_INVALID, "ark_write_batch: bad item");
      hoff.push_back(hdr.size());
      hdr.insert(hdr.end(), it.id, it.id + strlen(it.id));
      hdr.push_back(' ');
      const char tag[] = {'\0', 'B', 'F', 'M', ' ', 4};
      hdr.insert(hdr.end(), tag, tag + 6);
      const char* r = (const char*)&it.rows;
      hdr.insert(hdr.end(), r, r + 4);
      hdr.push_back(4);
      const char* c = (const char*)&cols;
      hdr.insert(hdr.end(), c, c + 4);
    }
    hoff.push_back(hdr.size());
    iov.clear();
    size_t total = 0;
    for (size_t i = i0; i < i1; ++i) {
      const size_t hl = hoff[i - i0 + 1] - hoff[i - i0];
      iov.push_back({hdr.data() + hoff[i - i0], hl});
      const size_t dl = sizeof(float) * (size_t)items[i].rows * (size_t)cols;
      if (dl) iov.push_back({(void*)items[i].data, dl});
      // scp: the offset of the matrix (just after "<utt> ")
      if (w->scp && fprintf(w->scp, "%s %s:%lld\n", items[i].id, w->ark_abs.c_str(),
                            (long long)(pos + (off_t)total + (off_t)strlen(items[i].id) + 1)) < 0)
        return w->failed = true, fail(FDLP_E_IO, "scp write failed");
      total += hl + dl;
    }
    // reserve the blocks of this writev first (one allocation call instead of block by block as the
    // page cache fills; 10.2-10.7 -> 11.6-12.6 GB/s on the MI355X box's overlay, profiles/r05m_*); a
    // filesystem without fallocate just writes
    (void)fallocate(fd, FALLOC_FL_KEEP_SIZE, pos, (off_t)total);
    size_t k = 0;  // writev until every iovec is out (it may write partially)
    while (k < iov.size()) {
      const int cnt = (int)std::min<size_t>(iov.size() - k, IOV_MAX);
      const ssize_t got = writev(fd, iov.data() + k, cnt);
      if (got < 0) return w->failed = true, fail(FDLP_E_IO, "ark write failed");
      size_t left = (size_t)got;
      while (k < iov.size() && left >= iov[k].iov_len) left -= iov[k++].iov_len;
      if (left) {
        iov[k].iov_base = (char*)iov[k].iov_base + left;
        iov[k].iov_len -= left;
      }
    }
    pos += (off_t)total;
  }
  return FDLP_OK;
}
}  // namespace fdlp

extern "C" {

// Closes the files and renames <ark>.tmp / <scp>.tmp to their final names (a JOB's outputs appear
// only once complete); after a write failure the temporaries are removed instead.
int fdlp_ark_close(fdlp_ark_writer* w) {
  if (!w) return FDLP_OK;
  int rc = FDLP_OK;
  if (w->ark && fclose(w->ark) != 0) rc = fdlp::fail(FDLP_E_IO, "ark close failed");
  if (w->scp && fclose(w->scp) != 0) rc = fdlp::fail(FDLP_E_IO, "scp close failed");
  if (rc != FDLP_OK || w->failed) {
    remove(w->ark_tmp.c_str());
    if (w->scp) remove(w->scp_tmp.c_str());
    if (rc == FDLP_OK) rc = fdlp::fail(FDLP_E_IO, "ark/scp not written (an earlier write failed)");
  } else {
    if (rename(w->ark_tmp.c_str(), w->ark_path.c_str()) != 0)
      rc = fdlp::fail(FDLP_E_IO, "cannot rename " + w->ark_tmp);
    if (w->scp && rc == FDLP_OK && rename(w->scp_tmp.c_str(), w->scp_path.c_str()) != 0)
      rc = fdlp::fail(FDLP_E_IO, "cannot rename " + w->scp_tmp);
  }
  delete w;
  return rc;
}

// Closes the files and removes the temporaries: a JOB that fails part-way publishes nothing under the
// final names (the reference raises before dict2Ark, so it never writes an ark either).
int fdlp_ark_abort(fdlp_ark_writer* w) {
  if (!w) return FDLP_OK;
  if (w->ark) fclose(w->ark);
  if (w->scp) fclose(w->scp);
  remove(w->ark_tmp.c_str());
  if (w->scp) remove(w->scp_tmp.c_str());
  delete w;
  return FDLP_OK;
}

// ---------------------------------------------------------------------------------------------
// Kaldi matrix reader ("scp:" / "ark:" rspecifiers) and double-matrix object writer, for the
// compute-cmvn-stats drop-in (bin/compute-cmvn-stats).  Binary Kaldi format only (what copy-feats
// and this library's ark writer produce).
// ---------------------------------------------------------------------------------------------
struct fdlp_mat_reader {
  bool scp = false;
  FILE* list = nullptr;       // scp file, or the ark stream itself for "ark:"
  bool own_list = true;
  FILE* cur = nullptr;        // scp: the ark file currently open
  std::string cur_path;
  std::string key;
  std::vector<float> data;
  std::vector<double> dbuf;
};

static int read_matrix_body(FILE* f, const std::string& where, std::vector<float>& out, std::vector<double>& dbuf,
                            int32_t* rows, int32_t* cols) {
  char hdr[2];
  if (fread(hdr, 1, 2, f) != 2 || hdr[0] != '\0' || hdr[1] != 'B')
    return fdlp::fail(FDLP_E_IO, "expected a binary Kaldi object at " + where);
  char tok[4] = {0, 0, 0, 0};
  if (fread(tok, 1, 3, f) != 3) return fdlp::fail(FDLP_E_IO, "truncated matrix header at " + where);
  const bool is_f = !memcmp(tok, "FM ", 3), is_d = !memcmp(tok, "DM ", 3);
  if (!is_f && !is_d) {
    if (tok[0] == 'C' && tok[1] == 'M') return fdlp::fail(FDLP_E_IO, "compressed matrices are not supported (" + where + ")");
    return fdlp::fail(FDLP_E_IO, "not a float/double matrix at " + where);
  }
  char sz;
  int32_t r = 0, c = 0;
  if (fread(&sz, 1, 1, f) != 1 || sz != 4 || fread(&r, 4, 1, f) != 1 || fread(&sz, 1, 1, f) != 1 || sz != 4 ||
      fread(&c, 4, 1, f) != 1 || r < 0 || c < 0)
    return fdlp::fail(FDLP_E_IO, "bad matrix dimensions at " + where);
  const size_t n = (size_t)r * (size_t)c;
  out.resize(n);
  if (is_f) {
    if (n && fread(out.data(), sizeof(float), n, f) != n) return fdlp::fail(FDLP_E_IO, "truncated matrix at " + where);
  } else {
    dbuf.resize(n);
    if (n && fread(dbuf.data(), sizeof(double), n, f) != n) return fdlp::fail(FDLP_E_IO, "truncated matrix at " + where);
    for (size_t i = 0; i < n; ++i) out[i] = (float)dbuf[i];
  }
  *rows = r;
  *cols = c;
  return FDLP_OK;
}

int fdlp_mat_reader_open(const char* spec, fdlp_mat_reader** out) {
  if (!spec || !out) return fdlp::fail(FDLP_E_INVALID, "fdlp_mat_reader_open: bad args");
  std::string s(spec);
  // strip Kaldi rspecifier options ("scp,p:" etc.): keep the type before the first ',' or ':'
  const size_t colon = s.find(':');
  if (colon == std::string::npos) return fdlp::fail(FDLP_E_INVALID, "rspecifier must start with scp: or ark: (" + s + ")");
  std::string type = s.substr(0, colon), path = s.substr(colon + 1);
  type = type.substr(0, type.find(','));
  if (type != "scp" && type != "ark") return fdlp::fail(FDLP_E_INVALID, "unsupported rspecifier type " + type);
  auto* r = new (std::nothrow) fdlp_mat_reader;
  if (!r) return fdlp::fail(FDLP_E_NOMEM, "fdlp_mat_reader_open: out of memory");
  r->scp = type == "scp";
  if (path == "-") {
    r->list = stdin;
    r->own_list = false;
  } else {
    r->list = fopen(path.c_str(), r->scp ? "r" : "rb");
  }
  if (!r->list) {
    delete r;
    return fdlp::fail(FDLP_E_IO, "cannot open " + path);
  }
  *out = r;
  return FDLP_OK;
}

int fdlp_mat_reader_next(fdlp_mat_reader* r, const char** key, int32_t* rows, int32_t* cols, const float** data) {
  if (!r || !key || !rows || !cols || !data) return fdlp::fail(FDLP_E_INVALID, "fdlp_mat_reader_next: bad args");
  if (r->scp) {
    char line[65536];
    for (;;) {
      if (!fgets(line, sizeof line, r->list)) return 0;
      std::string l(line);
      while (!l.empty() && (l.back() == '\n' || l.back() == '\r' || l.back() == ' ' || l.back() == '\t')) l.pop_back();
      size_t a = l.find_first_not_of(" \t");
      if (a == std::string::npos) continue;  // blank line
      size_t b = l.find_first_of(" \t", a);
      if (b == std::string::npos) return fdlp::fail(FDLP_E_IO, "bad scp line: " + l);
      r->key = l.substr(a, b - a);
      std::string rx = l.substr(l.find_first_not_of(" \t", b));
      std::string file = rx;
      long off = -1;
      const size_t c = rx.rfind(':');
      if (c != std::string::npos && c + 1 < rx.size() && rx.find_first_not_of("0123456789", c + 1) == std::string::npos) {
        file = rx.substr(0, c);
        off = atol(rx.c_str() + c + 1);
      }
      if (!r->cur || file != r->cur_path) {
        if (r->cur) fclose(r->cur);
        r->cur = fopen(file.c_str(), "rb");
        r->cur_path = file;
        if (!r->cur) return fdlp::fail(FDLP_E_IO, "cannot open " + file);
      }
      if (fseek(r->cur, off < 0 ? 0 : off, SEEK_SET) != 0) return fdlp::fail(FDLP_E_IO, "cannot seek in " + file);
      int rc = read_matrix_body(r->cur, rx, r->data, r->dbuf, rows, cols);
      if (rc != FDLP_OK) return rc;
      break;
    }
  } else {
    // "<key> " then the binary object
    std::string k;
    int ch;
    while ((ch = fgetc(r->list)) != EOF && (ch == ' ' || ch == '\n' || ch == '\t' || ch == '\r')) {}
    if (ch == EOF) return 0;
    do { k.push_back((char)ch); } while ((ch = fgetc(r->list)) != EOF && ch != ' ');
    if (ch == EOF) return fdlp::fail(FDLP_E_IO, "truncated ark after key " + k);
    r->key = k;
    int rc = read_matrix_body(r->list, "ark key " + k, r->data, r->dbuf, rows, cols);
    if (rc != FDLP_OK) return rc;
  }
  *key = r->key.c_str();
  *data = r->data.data();
  return 1;
}

int fdlp_mat_reader_close(fdlp_mat_reader* r) {
  if (!r) return FDLP_OK;
  if (r->cur) fclose(r->cur);
  if (r->list && r->own_list) fclose(r->list);
  delete r;
  return FDLP_OK;
}

int fdlp_kaldi_write_dmatrix(const char* path, const double* m, int32_t rows, int32_t cols, int32_t binary) {
  if (!path || rows < 0 || cols < 0 || (rows * (int64_t)cols > 0 && !m))
    return fdlp::fail(FDLP_E_INVALID, "fdlp_kaldi_write_dmatrix: bad args");
  FILE* f = fopen(path, binary ? "wb" : "w");
  if (!f) return fdlp::fail(FDLP_E_IO, std::string("cannot open ") + path);
  int ok = 1;
  if (binary) {
    const char hdr[] = {'\0', 'B', 'D', 'M', ' '};
    const char four = 4;
    ok &= fwrite(hdr, 1, 5, f) == 5;
    ok &= fwrite(&four, 1, 1, f) == 1;
    ok &= fwrite(&rows, 4, 1, f) == 1;
    ok &= fwrite(&four, 1, 1, f) == 1;
    ok &= fwrite(&cols, 4, 1, f) == 1;
    const size_t n = (size_t)rows * (size_t)cols;
    if (n) ok &= fwrite(m, sizeof(double), n, f) == n;
  } else if (cols == 0 || rows == 0) {
    ok &= fputs(" [ ]\n", f) >= 0;
  } else {  // Kaldi MatrixBase::Write text mode
    ok &= fputs(" [", f) >= 0;
    for (int32_t i = 0; i < rows; ++i) {
      ok &= fputs("\n  ", f) >= 0;
      for (int32_t j = 0; j < cols; ++j) ok &= fprintf(f, "%g ", m[(size_t)i * cols + j]) >= 0;
    }
    ok &= fputs("]\n", f) >= 0;
  }
  if (fclose(f) != 0) ok = 0;
  return ok ? FDLP_OK : fdlp::fail(FDLP_E_IO, std::string("write failed: ") + path);
}

}  // extern "C"
