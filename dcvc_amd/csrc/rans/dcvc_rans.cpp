// libdcvc_rans — host rANS entropy coder behind the C ABI in include/dcvc_rans.h.
//
// Behaviour follows the reference coders (DCVC-DC/src/cpp/rans/rans.cpp,
// DCVC-DC/src/cpp/py_rans/py_rans.cpp, DCVC-HEM/src/cpp/rans/rans_interface.cpp)
// so that streams are byte-identical; the implementation is organised for
// throughput instead:
//   * a CDF table is uploaded once (dcvc_cdf_table) instead of being copied on
//     every call, and carries a 2^LUT_BITS-entry lookup per distribution so the
//     decoder finds a symbol in O(1) instead of the reference's linear
//     std::find_if over the CDF (rans.cpp:295-298);
//   * symbols are resolved to (start, freq) pairs at encode time into one flat
//     buffer per stream part, flushed in reverse in a single tight loop;
//   * every input is validated before any state changes; malformed streams
//     stop with DCVC_ESTREAM instead of reading past the buffer.
#include "../../../include/dcvc_rans.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <numeric>
#include <thread>
#include <vector>

namespace {

constexpr uint32_t kPrecision = 16;             // probability bits (rans.cpp:27)
constexpr uint64_t kRansL = 1ull << 31;         // rANS64 lower bound
constexpr uint32_t kBypassBits = 4;             // rans.cpp:29
constexpr uint32_t kBypassMax = (1u << kBypassBits) - 1;
constexpr int kLutBits = 10;
constexpr uint32_t kMaxRawBypass = 1u << 28;    // keeps the bypass loop defined

// ---------------------------------------------------------------- tables
struct CdfTable {
  int num = 0;
  int stride = 0;
  std::vector<int32_t> cdf;      // [num][stride]
  std::vector<int32_t> size;     // valid entries per row
  std::vector<int32_t> offset;   // symbol offset per row
  std::vector<uint16_t> lut;     // [num][1 << kLutBits] first candidate symbol

  bool build(const int32_t *cdfs, int n, int st, const int32_t *sizes,
             const int32_t *offs) {
    if (!cdfs || !sizes || !offs || n <= 0 || st <= 1) return false;
    num = n;
    stride = st;
    cdf.assign(cdfs, cdfs + (size_t)n * st);
    size.assign(sizes, sizes + n);
    offset.assign(offs, offs + n);
    lut.assign((size_t)n << kLutBits, 0);
    for (int t = 0; t < n; ++t) {
      const int sz = size[t];
      if (sz < 2 || sz > st || sz > 65535) return false;
      const int32_t *c = &cdf[(size_t)t * st];
      uint16_t *l = &lut[(size_t)t << kLutBits];
      int s = 0;
      for (uint32_t b = 0; b < (1u << kLutBits); ++b) {
        const uint32_t cum = b << (kPrecision - kLutBits);
        while (s + 1 < sz - 1 && (uint32_t)c[s + 1] <= cum) ++s;
        l[b] = (uint16_t)s;
      }
    }
    return true;
  }
};

// ---------------------------------------------------------------- symbols
struct Sym {            // one rANS step, mirrors RansSymbol (rans.h:36-40)
  uint16_t start;
  uint16_t range;
  uint8_t bypass;
};

// Resolve one (symbol, index) pair into rANS steps (rans.cpp:90-137).
// Returns DCVC_OK or DCVC_ERANGE; `out` is appended to.
inline int push_symbol(std::vector<Sym> &out, const CdfTable &t, int idx,
                       int64_t sym) {
  const int32_t *c = &t.cdf[(size_t)idx * t.stride];
  const int32_t max_value = t.size[idx] - 2;
  int64_t value = sym - (int64_t)t.offset[idx];
  uint64_t raw = 0;
  if (value < 0) {
    raw = (uint64_t)(-2 * value - 1);
    value = max_value;
  } else if (value >= max_value) {
    raw = (uint64_t)(2 * (value - max_value));
    value = max_value;
  }
  if (raw >= kMaxRawBypass) return DCVC_ERANGE;
  out.push_back({(uint16_t)c[value], (uint16_t)(c[value + 1] - c[value]), 0});
  if (value == max_value) {
    uint32_t nb = 0;
    while ((raw >> (nb * kBypassBits)) != 0) ++nb;
    uint32_t v = nb;
    while (v >= kBypassMax) {
      out.push_back({(uint16_t)kBypassMax, (uint16_t)(kBypassMax + 1), 1});
      v -= kBypassMax;
    }
    out.push_back({(uint16_t)v, (uint16_t)(v + 1), 1});
    for (uint32_t j = 0; j < nb; ++j) {
      const uint32_t piece = (uint32_t)(raw >> (j * kBypassBits)) & kBypassMax;
      out.push_back({(uint16_t)piece, (uint16_t)(piece + 1), 1});
    }
  }
  return DCVC_OK;
}

// rANS64 encode of the buffered steps, last step first (rans.cpp:141-168).
bool flush_syms(const std::vector<Sym> &syms, std::vector<uint8_t> &stream) {
  std::vector<uint32_t> words(syms.size() + 2);
  uint32_t *end = words.data() + words.size();
  uint32_t *p = end;
  uint64_t x = kRansL;
  for (size_t i = syms.size(); i-- > 0;) {
    const Sym &s = syms[i];
    if (!s.bypass) {
      const uint64_t f = s.range;
      if (f == 0) return false;
      if (x >= ((kRansL >> kPrecision) << 32) * f) {
        *--p = (uint32_t)x;
        x >>= 32;
      }
      const uint64_t q = x / f;
      x = (q << kPrecision) + (x - q * f) + s.start;
    } else {
      // Rans64EncPutBits (rans.cpp:37-55): freq = 2^(16-nbits)
      const uint64_t f = 1ull << (kPrecision - kBypassBits);
      if (x >= ((kRansL >> kPrecision) << 32) * f) {
        *--p = (uint32_t)x;
        x >>= 32;
      }
      x = (x << kBypassBits) | s.start;
    }
  }
  p -= 2;  // Rans64EncFlush
  p[0] = (uint32_t)x;
  p[1] = (uint32_t)(x >> 32);
  const size_t nbytes = (size_t)(end - p) * 4;
  stream.resize(nbytes);
  std::memcpy(stream.data(), p, nbytes);
  return true;
}

// ---------------------------------------------------------------- worker
class Worker {
 public:
  Worker() : th_([this] { loop(); }) {}
  ~Worker() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(std::move(f));
      ++pending_;
    }
    cv_.notify_all();
  }
  void wait_idle() {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return pending_ == 0; });
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
      {
        std::lock_guard<std::mutex> lk(mu_);
        --pending_;
      }
      done_cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<std::function<void()>> q_;
  int pending_ = 0;
  bool stop_ = false;
  std::thread th_;
};

struct EncPart {
  std::vector<Sym> syms;
  std::vector<uint8_t> stream;
  int status = DCVC_OK;
  bool flushed = false;
};

}  // namespace

struct dcvc_cdf_table {
  std::shared_ptr<CdfTable> t;
};

struct dcvc_rans_enc {
  int parts = 1;
  std::vector<EncPart> part;
  std::vector<std::unique_ptr<Worker>> workers;  // empty when synchronous
};

struct dcvc_rans_dec {
  int parts = 1;
  std::vector<std::vector<uint32_t>> words;  // per part
  std::vector<size_t> pos;                   // next word to read
  std::vector<uint64_t> state;
};

namespace {

template <typename T>
int validate_indexes(const T *idx, int64_t n, const CdfTable &t,
                     bool allow_negative) {
  for (int64_t i = 0; i < n; ++i) {
    const int64_t v = idx[i];
    if (v < 0) {
      if (!allow_negative) return DCVC_EINVAL;
      continue;
    }
    if (v >= t.num) return DCVC_EINVAL;
  }
  return DCVC_OK;
}

template <typename T>
int encode_slice(EncPart &p, const T *sym, const T *idx, int64_t n,
                 const CdfTable &t) {
  p.syms.reserve(p.syms.size() + (size_t)n + (size_t)n / 8);
  for (int64_t i = 0; i < n; ++i) {
    const int k = (int)idx[i];
    if (k < 0) continue;  // DC skip (rans.cpp:91-93)
    const int r = push_symbol(p.syms, t, k, (int64_t)sym[i]);
    if (r != DCVC_OK) return r;
  }
  return DCVC_OK;
}

template <typename T>
int enc_encode(dcvc_rans_enc *e, const T *symbols, const T *indexes, int64_t n,
               std::shared_ptr<CdfTable> tab, bool allow_negative) {
  if (!e || n < 0 || !tab || (n > 0 && (!symbols || !indexes)))
    return DCVC_EINVAL;
  int r = validate_indexes(indexes, n, *tab, allow_negative);
  if (r != DCVC_OK) return r;
  if (!allow_negative) {
    // HEM symbols: reject values the bypass coder cannot represent up front
    for (int64_t i = 0; i < n; ++i) {
      const CdfTable &t = *tab;
      const int k = (int)indexes[i];
      const int64_t v = (int64_t)symbols[i] - t.offset[k];
      const int64_t mv = t.size[k] - 2;
      const int64_t raw = v < 0 ? -2 * v - 1 : (v >= mv ? 2 * (v - mv) : 0);
      if (raw >= (int64_t)kMaxRawBypass) return DCVC_ERANGE;
    }
  }
  const int parts = e->parts;
  const int64_t each = n / parts;
  for (int i = 0; i < parts; ++i) {
    const int64_t off = i * each;
    const int64_t cnt = (i < parts - 1) ? each : n - each * (parts - 1);
    EncPart &p = e->part[i];
    p.flushed = false;
    if (e->workers.empty()) {
      r = encode_slice(p, symbols + off, indexes + off, cnt, *tab);
      if (r != DCVC_OK) return r;
    } else {
      auto s = std::make_shared<std::vector<T>>(symbols + off, symbols + off + cnt);
      auto x = std::make_shared<std::vector<T>>(indexes + off, indexes + off + cnt);
      e->workers[i]->submit([&p, s, x, tab] {
        if (p.status != DCVC_OK) return;
        p.status = encode_slice(p, s->data(), x->data(), (int64_t)s->size(), *tab);
      });
    }
  }
  return DCVC_OK;
}

std::shared_ptr<CdfTable> make_table(const int32_t *cdfs, int cdf_num,
                                     int cdf_stride, const int32_t *sizes,
                                     const int32_t *offsets) {
  auto t = std::make_shared<CdfTable>();
  if (!t->build(cdfs, cdf_num, cdf_stride, sizes, offsets)) return nullptr;
  return t;
}

// Decode one slice of one part (rans.cpp:272-331 / rans_interface.cpp:184-244).
template <typename TI, typename TO>
int decode_slice(dcvc_rans_dec *d, int part, const TI *idx, int64_t n,
                 const CdfTable &t, TO *out, bool dc_format) {
  const std::vector<uint32_t> &w = d->words[part];
  size_t pos = d->pos[part];
  uint64_t x = d->state[part];
  const size_t nw = w.size();
  bool bad = false;
  auto next_word = [&]() -> uint32_t {
    if (pos >= nw) {
      bad = true;
      return 0;
    }
    return w[pos++];
  };
  const uint32_t mask = (1u << kPrecision) - 1;
  for (int64_t i = 0; i < n; ++i) {
    const int k = (int)idx[i];
    if (k < 0) {  // only reachable in DC format; reference reads offsets[-1]
      out[i] = 0;
      continue;
    }
    const int32_t *c = &t.cdf[(size_t)k * t.stride];
    const int32_t max_value = t.size[k] - 2;
    const uint32_t cum = (uint32_t)(x & mask);
    int s = t.lut[((size_t)k << kLutBits) + (cum >> (kPrecision - kLutBits))];
    while (s < max_value && (uint32_t)c[s + 1] <= cum) ++s;
    const uint64_t start = (uint32_t)c[s];
    const uint64_t freq = (uint32_t)(c[s + 1] - c[s]);
    x = freq * (x >> kPrecision) + (x & mask) - start;
    if (x < kRansL) x = (x << 32) | next_word();
    int64_t value = s;
    if (value == max_value) {
      auto get_bits = [&]() -> uint32_t {
        const uint32_t v = (uint32_t)(x & kBypassMax);
        x >>= kBypassBits;
        if (x < kRansL) x = (x << 32) | next_word();
        return v;
      };
      uint32_t v = get_bits();
      uint32_t nb = v;
      while (v == kBypassMax && !bad) {
        v = get_bits();
        nb += v;
        if (nb > 8) break;
      }
      if (nb > 7) return DCVC_ESTREAM;
      uint32_t raw = 0;
      for (uint32_t j = 0; j < nb; ++j) raw |= get_bits() << (j * kBypassBits);
      value = raw >> 1;
      if (raw & 1)
        value = -value - 1;
      else
        value += max_value;
    }
    if (bad) return DCVC_ESTREAM;
    const int64_t res = value + t.offset[k];
    out[i] = dc_format ? (TO)(int16_t)res : (TO)res;
  }
  d->pos[part] = pos;
  d->state[part] = x;
  return DCVC_OK;
}

template <typename TI, typename TO>
int dec_decode(dcvc_rans_dec *d, const TI *indexes, int64_t n,
               const CdfTable &t, TO *out, bool dc_format) {
  if (!d || n < 0 || (n > 0 && (!indexes || !out))) return DCVC_EINVAL;
  if (d->words.empty()) return DCVC_EINVAL;
  int r = validate_indexes(indexes, n, t, dc_format);
  if (r != DCVC_OK) return r;
  const int parts = d->parts;
  const int64_t each = n / parts;
  if (parts == 1) return decode_slice(d, 0, indexes, n, t, out, dc_format);
  std::vector<int> status(parts, DCVC_OK);
  std::vector<std::thread> th;
  for (int i = 0; i < parts; ++i) {
    const int64_t off = i * each;
    const int64_t cnt = (i < parts - 1) ? each : n - each * (parts - 1);
    th.emplace_back([=, &status, &t] {
      status[i] = decode_slice(d, i, indexes + off, cnt, t, out + off, dc_format);
    });
  }
  for (auto &x : th) x.join();
  for (int s : status)
    if (s != DCVC_OK) return s;
  return DCVC_OK;
}

int parse_into(dcvc_rans_dec *d, int part, const uint8_t *p, int64_t len) {
  if (len < 8 || (len & 3)) return DCVC_ESTREAM;
  std::vector<uint32_t> &w = d->words[part];
  w.resize((size_t)len / 4);
  std::memcpy(w.data(), p, (size_t)len);
  d->state[part] = (uint64_t)w[0] | ((uint64_t)w[1] << 32);  // Rans64DecInit
  d->pos[part] = 2;
  return DCVC_OK;
}

}  // namespace

extern "C" {

int dcvc_pmf_to_quantized_cdf(const float *pmf, int n, int precision,
                              uint32_t *cdf_out) {
  // Restates ops.cpp:24-82: round to counts, renormalise to 2^precision,
  // prefix-sum, then give every empty bin one count taken from the
  // smallest bin that can spare it.
  if (!pmf || !cdf_out || n <= 0 || precision <= 0 || precision > 24)
    return DCVC_EINVAL;
  const size_t m = (size_t)n + 1;
  std::vector<uint32_t> c(m);
  c[0] = 0;
  for (int i = 0; i < n; ++i) {
    const float scaled = pmf[i] * (float)(1 << precision);
    c[i + 1] = static_cast<uint32_t>(std::round(scaled) + 0.5);
  }
  uint32_t total = 0;
  for (uint32_t v : c) total += v;
  if (total == 0) return DCVC_EINVAL;
  for (auto &v : c)
    v = static_cast<uint32_t>(((1ull << precision) * (uint64_t)v) / total);
  for (size_t i = 1; i < m; ++i) c[i] += c[i - 1];
  c[m - 1] = 1u << precision;
  for (size_t i = 0; i + 1 < m; ++i) {
    if (c[i] != c[i + 1]) continue;
    uint32_t best = ~0u;
    long steal = -1;
    for (size_t j = 0; j + 1 < m; ++j) {
      const uint32_t f = c[j + 1] - c[j];
      if (f > 1 && f < best) {
        best = f;
        steal = (long)j;
      }
    }
    if (steal < 0) return DCVC_EINVAL;
    if ((size_t)steal < i) {
      for (size_t j = (size_t)steal + 1; j <= i; ++j) c[j]--;
    } else {
      for (size_t j = i + 1; j <= (size_t)steal; ++j) c[j]++;
    }
  }
  std::memcpy(cdf_out, c.data(), m * sizeof(uint32_t));
  return DCVC_OK;
}

dcvc_cdf_table *dcvc_cdf_table_create(const int32_t *cdfs, int cdf_num,
                                      int cdf_stride, const int32_t *cdf_sizes,
                                      const int32_t *offsets) {
  auto t = make_table(cdfs, cdf_num, cdf_stride, cdf_sizes, offsets);
  if (!t) return nullptr;
  auto *h = new (std::nothrow) dcvc_cdf_table;
  if (h) h->t = std::move(t);
  return h;
}

void dcvc_cdf_table_destroy(dcvc_cdf_table *t) { delete t; }

dcvc_rans_enc *dcvc_rans_enc_create(int multithread, int stream_part) {
  if (stream_part < 1 || stream_part > 16) return nullptr;
  auto *e = new (std::nothrow) dcvc_rans_enc;
  if (!e) return nullptr;
  e->parts = stream_part;
  e->part.resize(stream_part);
  // reference: multiThread || streamPart > 1 selects the threaded encoder
  if (multithread || stream_part > 1)
    for (int i = 0; i < stream_part; ++i)
      e->workers.emplace_back(new Worker());
  return e;
}

void dcvc_rans_enc_destroy(dcvc_rans_enc *e) { delete e; }

int dcvc_rans_enc_encode_with_indexes_i16(dcvc_rans_enc *e,
                                          const int16_t *symbols,
                                          const int16_t *indexes, int64_t n,
                                          const int32_t *cdfs, int cdf_num,
                                          int cdf_stride,
                                          const int32_t *cdf_sizes,
                                          const int32_t *offsets) {
  auto t = make_table(cdfs, cdf_num, cdf_stride, cdf_sizes, offsets);
  if (!t) return DCVC_EINVAL;
  return enc_encode(e, symbols, indexes, n, t, true);
}

int dcvc_rans_enc_encode_table_i16(dcvc_rans_enc *e, const int16_t *symbols,
                                   const int16_t *indexes, int64_t n,
                                   const dcvc_cdf_table *t) {
  if (!t) return DCVC_EINVAL;
  return enc_encode(e, symbols, indexes, n, t->t, true);
}

int dcvc_rans_enc_encode_table_i32(dcvc_rans_enc *e, const int32_t *symbols,
                                   const int32_t *indexes, int64_t n,
                                   const dcvc_cdf_table *t) {
  if (!t) return DCVC_EINVAL;
  return enc_encode(e, symbols, indexes, n, t->t, false);
}

int dcvc_rans_enc_flush(dcvc_rans_enc *e) {
  if (!e) return DCVC_EINVAL;
  for (int i = 0; i < e->parts; ++i) {
    EncPart &p = e->part[i];
    auto job = [&p] {
      if (p.status == DCVC_OK && !flush_syms(p.syms, p.stream))
        p.status = DCVC_EINVAL;
      p.flushed = true;
    };
    if (e->workers.empty())
      job();
    else
      e->workers[i]->submit(job);
  }
  if (e->workers.empty()) {
    for (auto &p : e->part)
      if (p.status != DCVC_OK) return p.status;
  }
  return DCVC_OK;
}

static int enc_wait(dcvc_rans_enc *e) {
  for (auto &w : e->workers) w->wait_idle();
  for (auto &p : e->part) {
    if (p.status != DCVC_OK) return p.status;
    if (!p.flushed) return DCVC_EBUSY;
  }
  return DCVC_OK;
}

static int header_bytes(const dcvc_rans_enc *e, int *per) {
  size_t maxsz = 0;
  for (int i = 0; i + 1 < e->parts; ++i)
    maxsz = std::max(maxsz, e->part[i].stream.size());
  *per = maxsz > 65535 ? 4 : 2;
  return 1 + (e->parts > 1 ? (e->parts - 1) * *per : 0);
}

int64_t dcvc_rans_enc_stream_size(dcvc_rans_enc *e, int with_header) {
  if (!e) return DCVC_EINVAL;
  int r = enc_wait(e);
  if (r != DCVC_OK) return r;
  if (!with_header && e->parts != 1) return DCVC_EINVAL;
  int64_t total = 0;
  for (auto &p : e->part) total += (int64_t)p.stream.size();
  if (with_header) {
    int per;
    total += header_bytes(e, &per);
  }
  return total;
}

int64_t dcvc_rans_enc_get_stream(dcvc_rans_enc *e, int with_header,
                                 uint8_t *out, int64_t cap) {
  const int64_t need = dcvc_rans_enc_stream_size(e, with_header);
  if (need < 0) return need;
  if (!out || cap < need) return DCVC_EINVAL;
  uint8_t *o = out;
  if (with_header) {
    int per;
    const int hb = header_bytes(e, &per);
    o[0] = (uint8_t)(((e->parts - 1) << 4) + (per == 2 ? 1 : 0));
    for (int i = 0; i + 1 < e->parts; ++i) {
      const uint32_t sz = (uint32_t)e->part[i].stream.size();
      for (int b = 0; b < per; ++b) o[1 + per * i + b] = (uint8_t)(sz >> (8 * b));
    }
    o += hb;
  }
  for (auto &p : e->part) {
    std::memcpy(o, p.stream.data(), p.stream.size());
    o += p.stream.size();
  }
  return need;
}

int dcvc_rans_enc_reset(dcvc_rans_enc *e) {
  if (!e) return DCVC_EINVAL;
  for (auto &w : e->workers) w->wait_idle();
  for (auto &p : e->part) {
    p.syms.clear();
    p.status = DCVC_OK;
    p.flushed = false;
  }
  return DCVC_OK;
}

dcvc_rans_dec *dcvc_rans_dec_create(int stream_part) {
  if (stream_part < 1 || stream_part > 16) return nullptr;
  auto *d = new (std::nothrow) dcvc_rans_dec;
  if (!d) return nullptr;
  d->parts = stream_part;
  return d;
}

void dcvc_rans_dec_destroy(dcvc_rans_dec *d) { delete d; }

int dcvc_rans_dec_set_stream(dcvc_rans_dec *d, const uint8_t *data,
                             int64_t len, int with_header) {
  if (!d || !data || len <= 0) return DCVC_EINVAL;
  d->words.assign(d->parts, {});
  d->pos.assign(d->parts, 0);
  d->state.assign(d->parts, 0);
  if (!with_header) {
    if (d->parts != 1) return DCVC_EINVAL;
    return parse_into(d, 0, data, len);
  }
  const uint8_t flag = data[0];
  const int nstreams = (flag >> 4) + 1;
  if (nstreams != d->parts) return DCVC_ESTREAM;
  const int per = (flag & 0x0f) == 1 ? 2 : 4;
  int64_t off = 1, total = 0;
  std::vector<int64_t> sizes;
  for (int i = 0; i + 1 < nstreams; ++i) {
    if (off + per > len) return DCVC_ESTREAM;
    uint32_t s = 0;
    for (int b = 0; b < per; ++b) s |= (uint32_t)data[off + b] << (8 * b);
    off += per;
    sizes.push_back(s);
    total += s;
  }
  sizes.push_back(len - off - total);
  for (int i = 0; i < nstreams; ++i) {
    if (sizes[i] < 0 || off + sizes[i] > len) return DCVC_ESTREAM;
    int r = parse_into(d, i, data + off, sizes[i]);
    if (r != DCVC_OK) return r;
    off += sizes[i];
  }
  return DCVC_OK;
}

int dcvc_rans_dec_decode_with_indexes_i16(dcvc_rans_dec *d,
                                          const int16_t *indexes, int64_t n,
                                          const int32_t *cdfs, int cdf_num,
                                          int cdf_stride,
                                          const int32_t *cdf_sizes,
                                          const int32_t *offsets,
                                          int16_t *out) {
  auto t = make_table(cdfs, cdf_num, cdf_stride, cdf_sizes, offsets);
  if (!t) return DCVC_EINVAL;
  return dec_decode(d, indexes, n, *t, out, true);
}

int dcvc_rans_dec_decode_table_i16(dcvc_rans_dec *d, const int16_t *indexes,
                                   int64_t n, const dcvc_cdf_table *t,
                                   int16_t *out) {
  if (!t) return DCVC_EINVAL;
  return dec_decode(d, indexes, n, *t->t, out, true);
}

int dcvc_rans_dec_decode_table_i32(dcvc_rans_dec *d, const int32_t *indexes,
                                   int64_t n, const dcvc_cdf_table *t,
                                   int32_t *out) {
  if (!t) return DCVC_EINVAL;
  return dec_decode(d, indexes, n, *t->t, out, false);
}

}  // extern "C"
