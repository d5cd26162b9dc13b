// libdcvc_rans — host rANS entropy coder behind the C ABI in include/dcvc_rans.h.
//
// Behaviour follows the reference coders (DCVC-DC/src/cpp/rans/rans.cpp,
// DCVC-DC/src/cpp/py_rans/py_rans.cpp, DCVC-HEM/src/cpp/rans/rans_interface.cpp)
// so that streams are byte-identical; the implementation is organised for
// throughput instead:
//   * a CDF table is uploaded once (dcvc_cdf_table) instead of being copied on
//     every call.  It carries, per (row, symbol), the encoder's reciprocal
//     step (ryg_rans' Rans64EncSymbol construction: x / f becomes a 64x64
//     mul-high and a shift, exact for every x < 2^64) and, per row, a
//     2^LUT_BITS-entry lookup so the decoder finds a symbol in O(1) instead of
//     the reference's linear std::find_if over the CDF (rans.cpp:295-298);
//   * encode calls only copy + validate their slice of symbols (in parallel,
//     one task per stream part); flush walks every part's symbols last to
//     first and resolves CDF entries and bypass escapes inline, so no
//     intermediate step list is built;
//   * stream parts are encoded and decoded on a persistent thread pool (one
//     task per part) instead of a thread spawned per call;
//   * every input is validated before any state changes; malformed streams
//     stop with DCVC_ESTREAM instead of reading past the buffer.
#include "../../../include/dcvc_rans.h"

#include <algorithm>
#include <cstdlib>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

namespace {

constexpr uint32_t kPrecision = 16;             // probability bits (rans.cpp:27)
constexpr uint64_t kRansL = 1ull << 31;         // rANS64 lower bound
constexpr uint32_t kBypassBits = 4;             // rans.cpp:29
constexpr uint32_t kBypassMax = (1u << kBypassBits) - 1;
constexpr int kLutBits = 7;
constexpr uint32_t kMaxRawBypass = 1u << 28;    // keeps the bypass loop defined
constexpr int kMaxStepsPerSymbol = 12;          // 1 + count steps + 7 pieces, rounded up

// ---------------------------------------------------------------- tables
struct EncStep {        // one precomputed rANS encode step (start, freq)
  uint64_t rcp;         // reciprocal of freq (mul-high operand)
  uint32_t bias;        // start, or start + 2^16 - 1 when freq == 1
  uint16_t freq;
  uint8_t shift;
  uint8_t pad;
};

struct Row {
  int32_t offset;       // symbol offset
  int32_t maxv;         // cdf_size - 2: the escape symbol
};

struct CdfTable {
  int num = 0;
  int stride = 0;
  std::vector<int32_t> cdf;      // [num][stride], the caller's table
  std::vector<Row> row;          // [num]
  std::vector<uint32_t> packed;  // [num][stride] cdf[s] | (cdf[s+1]-cdf[s]) << 16
  std::vector<EncStep> enc;      // [num][stride]
  std::vector<uint16_t> lut;     // [num][1 << kLutBits] first candidate symbol

  bool build(const int32_t *cdfs, int n, int st, const int32_t *sizes,
             const int32_t *offs) {
    if (!cdfs || !sizes || !offs || n <= 0 || st <= 1) return false;
    num = n;
    stride = st;
    cdf.assign(cdfs, cdfs + (size_t)n * st);
    row.resize(n);
    packed.assign((size_t)n * st, 0);
    enc.assign((size_t)n * st, EncStep{});
    lut.assign((size_t)n << kLutBits, 0);
    for (int t = 0; t < n; ++t) {
      const int sz = sizes[t];
      if (sz < 2 || sz > st || sz > 65535) return false;
      row[t] = {offs[t], sz - 2};
      const int32_t *c = &cdf[(size_t)t * st];
      for (int s = 0; s + 1 < sz; ++s) {
        const int64_t start = c[s], freq = (int64_t)c[s + 1] - c[s];
        // a step the coder can take: 0 <= start, 0 < freq, start + freq <= 2^16
        if (start < 0 || freq <= 0 || start + freq > (1 << kPrecision) || freq >= (1 << kPrecision)) {
          // The reference accepts any table and misbehaves on such a step at
          // coding time; here the step is marked unusable (freq 0) and
          // coding a symbol that needs it fails with DCVC_EINVAL.
          enc[(size_t)t * st + s] = EncStep{0, 0, 0, 0, 0};
          packed[(size_t)t * st + s] = (uint32_t)(start & 0xffff);
          continue;
        }
        packed[(size_t)t * st + s] = (uint32_t)start | ((uint32_t)freq << 16);
        EncStep &e = enc[(size_t)t * st + s];
        e.freq = (uint16_t)freq;
        if (freq < 2) {
          e.rcp = ~0ull;
          e.shift = 0;
          e.bias = (uint32_t)(start + (1 << kPrecision) - 1);
        } else {
          uint32_t shift = 0;
          while ((uint64_t)freq > (1ull << shift)) ++shift;
          uint64_t x0 = (uint64_t)freq - 1, x1 = 1ull << (shift + 31);
          const uint64_t t1 = x1 / (uint64_t)freq;
          x0 += (x1 % (uint64_t)freq) << 32;
          const uint64_t t0 = x0 / (uint64_t)freq;
          e.rcp = t0 + (t1 << 32);
          e.shift = (uint8_t)(shift - 1);
          e.bias = (uint32_t)start;
        }
      }
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

// ---------------------------------------------------------------- pool
// One process-wide pool of persistent worker threads shared by every encoder
// and decoder (several GOP lanes, each with an I- and a P-codec, would
// otherwise each keep stream_part - 1 threads: 84 per process at 3 lanes x 4
// coder objects x 7).  run(tasks, fn) queues a batch, works on it on the
// calling thread too, and returns when all of its tasks are done; batches of
// concurrent callers are served in arrival order.  Workers default to
// min(15, hardware threads - 1), set by dcvc_rans_set_threads (or the
// DCVC_CODER_THREADS environment variable) before the first coder call.
class Pool {
 public:
  static Pool &shared() {
    static Pool p(configured());
    return p;
  }
  static int configured() {
    int n = g_threads.load();
    if (n < 0) {
      const char *e = std::getenv("DCVC_CODER_THREADS");
      n = e ? std::atoi(e) : -1;
    }
    if (n < 0) {
      const int hw = (int)std::thread::hardware_concurrency();
      n = std::min(15, std::max(0, hw - 1));
    }
    return std::min(n, 64);
  }
  static std::atomic<int> g_threads;
  static std::atomic<bool> g_started;
  int workers() const { return (int)th_.size(); }

  void run(int tasks, const std::function<void(int)> &fn) {
    if (tasks <= 0) return;
    if (th_.empty() || tasks == 1) {
      for (int i = 0; i < tasks; ++i) fn(i);
      return;
    }
    Batch b;
    b.fn = &fn;
    b.tasks = tasks;
    b.remaining = tasks;
    std::unique_lock<std::mutex> lk(mu_);
    q_.push_back(&b);
    lk.unlock();
    cv_.notify_all();
    int i;
    for (;;) {
      lk.lock();
      const bool got = claim(&b, &i);
      lk.unlock();
      if (!got) break;
      fn(i);
      lk.lock();
      --b.remaining;
      lk.unlock();
    }
    lk.lock();
    b.done.wait(lk, [&b] { return b.remaining == 0; });
  }

 private:
  struct Batch {
    const std::function<void(int)> *fn = nullptr;
    int tasks = 0, next = 0, remaining = 0;
    std::condition_variable done;
  };
  explicit Pool(int workers) {
    g_started = true;
    for (int i = 0; i < workers; ++i) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
  }
  // under mu_: the next task of b; a batch with none left leaves the queue
  // (so no worker can reach it after its caller has returned)
  bool claim(Batch *b, int *idx) {
    if (b->next < b->tasks) {
      *idx = b->next++;
      if (b->next == b->tasks) q_.erase(std::remove(q_.begin(), q_.end(), b), q_.end());
      return true;
    }
    return false;
  }
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
      if (stop_) return;
      Batch *b = q_.front();
      int i;
      if (!claim(b, &i)) continue;
      lk.unlock();
      (*b->fn)(i);
      lk.lock();
      if (--b->remaining == 0) b->done.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Batch *> q_;
  bool stop_ = false;
};
std::atomic<int> Pool::g_threads{-1};
std::atomic<bool> Pool::g_started{false};

// ---------------------------------------------------------------- encoder
struct Record {                      // one encode call's slice of a part
  std::shared_ptr<CdfTable> tab;
  size_t off, n;
};

struct EncPart {
  std::vector<int32_t> sym, idx;     // every buffered symbol / index, call order
  std::vector<Record> rec;
  std::unique_ptr<uint32_t[]> words; // flush output, written downwards
  size_t cap = 0;
  size_t begin = 0;                  // stream = words[begin, cap)
  int status = DCVC_OK;
  bool flushed = false;
};

inline uint64_t mulhi64(uint64_t a, uint64_t b) {
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
}

// rANS64 encode of one part, last symbol first (rans.cpp:141-168 on the step
// list rans.cpp:90-137 would have built).  Bypass escapes of a symbol are
// taken in reverse: raw pieces high to low, then the count steps, then the
// symbol's own escape step.
int flush_part(EncPart &p) {
  size_t bound = 2;
  for (const Record &r : p.rec) bound += r.n * kMaxStepsPerSymbol;
  if (bound > p.cap) {
    p.words.reset(new (std::nothrow) uint32_t[bound]);
    if (!p.words) {
      p.cap = 0;
      return DCVC_ENOMEM;
    }
    p.cap = bound;
  }
  uint32_t *const end = p.words.get() + p.cap;
  uint32_t *o = end;
  uint64_t x = kRansL;
  constexpr uint64_t kXmaxUnit = (kRansL >> kPrecision) << 32;
  auto put_bits = [&](uint32_t v) {
    if (x >= (kXmaxUnit << (kPrecision - kBypassBits))) {
      *--o = (uint32_t)x;
      x >>= 32;
    }
    x = (x << kBypassBits) | v;
  };
  for (size_t ri = p.rec.size(); ri-- > 0;) {
    const Record &r = p.rec[ri];
    const CdfTable &t = *r.tab;
    const int32_t *sym = p.sym.data() + r.off;
    const int32_t *idx = p.idx.data() + r.off;
    const Row *rows = t.row.data();
    const EncStep *steps = t.enc.data();
    const size_t st = (size_t)t.stride;
    for (size_t i = r.n; i-- > 0;) {
      const int k = idx[i];
      if (k < 0) continue;  // DC skip (rans.cpp:91-93)
      const Row rw = rows[k];
      int64_t value = (int64_t)sym[i] - rw.offset;
      if (value < 0 || value >= rw.maxv) {
        const uint64_t raw = value < 0 ? (uint64_t)(-2 * value - 1) : (uint64_t)(2 * (value - rw.maxv));
        uint32_t nb = 0;
        while ((raw >> (nb * kBypassBits)) != 0) ++nb;
        for (uint32_t j = nb; j-- > 0;) put_bits((uint32_t)(raw >> (j * kBypassBits)) & kBypassMax);
        put_bits(nb % kBypassMax);
        for (uint32_t c = nb / kBypassMax; c-- > 0;) put_bits(kBypassMax);
        value = rw.maxv;
      }
      const EncStep &e = steps[(size_t)k * st + (size_t)value];
      if (e.freq == 0) return DCVC_EINVAL;
      if (x >= kXmaxUnit * e.freq) {
        *--o = (uint32_t)x;
        x >>= 32;
      }
      const uint64_t q = mulhi64(x, e.rcp) >> e.shift;
      x += e.bias + q * ((1u << kPrecision) - e.freq);
    }
  }
  o -= 2;  // Rans64EncFlush
  o[0] = (uint32_t)x;
  o[1] = (uint32_t)(x >> 32);
  p.begin = (size_t)(o - p.words.get());
  return DCVC_OK;
}

// Copy + validate one part's slice of an encode call.
template <typename T>
int copy_slice(EncPart &p, const T *sym, const T *idx, size_t n, const CdfTable &t, bool dc) {
  const size_t o = p.sym.size();
  p.sym.resize(o + n);
  p.idx.resize(o + n);
  int32_t *ds = p.sym.data() + o, *di = p.idx.data() + o;
  const int num = t.num;
  for (size_t i = 0; i < n; ++i) {
    const int32_t k = (int32_t)idx[i];
    if (k >= num || (k < 0 && !dc)) return DCVC_EINVAL;
    ds[i] = (int32_t)sym[i];
    di[i] = k;
  }
  if (!dc) {
    // HEM symbols: reject values the bypass coder cannot represent up front
    // (the reference's bypass loop does not terminate on them)
    for (size_t i = 0; i < n; ++i) {
      const Row rw = t.row[di[i]];
      const int64_t v = (int64_t)ds[i] - rw.offset;
      const int64_t raw = v < 0 ? -2 * v - 1 : (v >= rw.maxv ? 2 * (v - rw.maxv) : 0);
      if (raw >= (int64_t)kMaxRawBypass) return DCVC_ERANGE;
    }
  }
  return DCVC_OK;
}

}  // namespace

struct dcvc_cdf_table {
  std::shared_ptr<CdfTable> t;
};

struct dcvc_rans_enc {
  int parts = 1;
  std::vector<EncPart> part;
  Pool *pool = nullptr;
  int status = DCVC_OK;   // first failure of an encode call since reset
};

struct dcvc_rans_dec {
  int parts = 1;
  std::vector<std::vector<uint32_t>> words;  // per part
  std::vector<size_t> pos;                   // next word to read
  std::vector<uint64_t> state;
  Pool *pool = nullptr;
};

namespace {

template <typename T>
int enc_encode(dcvc_rans_enc *e, const T *symbols, const T *indexes, int64_t n,
               std::shared_ptr<CdfTable> tab, bool dc) {
  if (!e || n < 0 || !tab || (n > 0 && (!symbols || !indexes))) return DCVC_EINVAL;
  const int parts = e->parts;
  const int64_t each = n / parts;
  std::vector<int> st(parts, DCVC_OK);
  std::vector<size_t> before(parts);
  for (int i = 0; i < parts; ++i) before[i] = e->part[i].sym.size();
  e->pool->run(parts, [&](int i) {
    const int64_t off = i * each;
    const int64_t cnt = (i < parts - 1) ? each : n - each * (parts - 1);
    st[i] = copy_slice(e->part[i], symbols + off, indexes + off, (size_t)cnt, *tab, dc);
  });
  for (int i = 0; i < parts; ++i) {
    if (st[i] != DCVC_OK) {
      // all-or-nothing: drop this call's symbols from every part
      for (int j = 0; j < parts; ++j) {
        e->part[j].sym.resize(before[j]);
        e->part[j].idx.resize(before[j]);
      }
      return st[i];
    }
  }
  for (int i = 0; i < parts; ++i) {
    EncPart &p = e->part[i];
    p.rec.push_back({tab, before[i], p.sym.size() - before[i]});
    p.flushed = false;
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
  const int num = t.num;
  const size_t st = (size_t)t.stride;
  const Row *rows = t.row.data();
  const uint32_t *packed = t.packed.data();
  const uint16_t *lut = t.lut.data();
  for (int64_t i = 0; i < n; ++i) {
    const int k = (int)idx[i];
    if (k < 0) {
      if (!dc_format) return DCVC_EINVAL;
      out[i] = 0;  // reference reads offsets[-1]; a skipped symbol decodes as 0
      continue;
    }
    if (k >= num) return DCVC_EINVAL;
    const uint32_t *c = packed + (size_t)k * st;
    const Row rw = rows[k];
    const uint32_t cum = (uint32_t)(x & mask);
    int s = lut[((size_t)k << kLutBits) + (cum >> (kPrecision - kLutBits))];
    while (s < rw.maxv && (c[s + 1] & 0xffff) <= cum) ++s;
    const uint32_t e = c[s];
    const uint64_t start = e & 0xffff, freq = e >> 16;
    x = freq * (x >> kPrecision) + (x & mask) - start;
    if (x < kRansL) x = (x << 32) | next_word();
    int64_t value = s;
    if (value == rw.maxv) {
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
        value += rw.maxv;
    }
    if (bad) return DCVC_ESTREAM;
    const int64_t res = value + rw.offset;
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
  // indexes are checked up front so a bad call leaves the decoder untouched
  for (int64_t i = 0; i < n; ++i) {
    const int64_t v = indexes[i];
    if (v >= t.num || (v < 0 && !dc_format)) return DCVC_EINVAL;
  }
  const int parts = d->parts;
  const int64_t each = n / parts;
  if (parts == 1) return decode_slice(d, 0, indexes, n, t, out, dc_format);
  std::vector<int> status(parts, DCVC_OK);
  d->pool->run(parts, [&](int i) {
    const int64_t off = i * each;
    const int64_t cnt = (i < parts - 1) ? each : n - each * (parts - 1);
    status[i] = decode_slice(d, i, indexes + off, cnt, t, out + off, dc_format);
  });
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
  // (py_rans.cpp:11-20); here the parts are worked on by the process-wide
  // pool plus the caller.  The stream is the same either way.
  (void)multithread;
  e->pool = &Pool::shared();
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
  e->pool->run(e->parts, [e](int i) {
    EncPart &p = e->part[i];
    p.status = flush_part(p);
    p.flushed = true;
  });
  for (auto &p : e->part)
    if (p.status != DCVC_OK) return p.status;
  return DCVC_OK;
}

static int enc_ready(dcvc_rans_enc *e) {
  for (auto &p : e->part) {
    if (p.status != DCVC_OK) return p.status;
    if (!p.flushed) return DCVC_EBUSY;
  }
  return DCVC_OK;
}

static size_t part_bytes(const EncPart &p) { return (p.cap - p.begin) * 4; }

static int header_bytes(const dcvc_rans_enc *e, int *per) {
  size_t maxsz = 0;
  for (int i = 0; i + 1 < e->parts; ++i) maxsz = std::max(maxsz, part_bytes(e->part[i]));
  *per = maxsz > 65535 ? 4 : 2;
  return 1 + (e->parts > 1 ? (e->parts - 1) * *per : 0);
}

int64_t dcvc_rans_enc_stream_size(dcvc_rans_enc *e, int with_header) {
  if (!e) return DCVC_EINVAL;
  int r = enc_ready(e);
  if (r != DCVC_OK) return r;
  if (!with_header && e->parts != 1) return DCVC_EINVAL;
  int64_t total = 0;
  for (auto &p : e->part) total += (int64_t)part_bytes(p);
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
      const uint32_t sz = (uint32_t)part_bytes(e->part[i]);
      for (int b = 0; b < per; ++b) o[1 + per * i + b] = (uint8_t)(sz >> (8 * b));
    }
    o += hb;
  }
  for (auto &p : e->part) {
    std::memcpy(o, p.words.get() + p.begin, part_bytes(p));
    o += part_bytes(p);
  }
  return need;
}

int dcvc_rans_enc_reset(dcvc_rans_enc *e) {
  if (!e) return DCVC_EINVAL;
  for (auto &p : e->part) {
    p.sym.clear();
    p.idx.clear();
    p.rec.clear();
    p.begin = p.cap;
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
  d->pool = &Pool::shared();
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

int dcvc_rans_set_threads(int workers) {
  if (workers < 0 || workers > 64) return DCVC_EINVAL;
  if (Pool::g_started.load()) return Pool::shared().workers() == workers ? DCVC_OK : DCVC_EBUSY;
  Pool::g_threads = workers;
  return DCVC_OK;
}

int dcvc_rans_threads(void) { return Pool::shared().workers(); }
