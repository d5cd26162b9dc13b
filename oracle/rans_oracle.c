/*
 * rans_oracle.c — TEST INFRASTRUCTURE ONLY (CPU oracle).  Never linked into,
 * loaded by, or called from the product path (dcvc_amd/); only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
 *
 * A deliberately plain C restatement of the reference entropy coder, written
 * for readability, with the reference's linear CDF search:
 *   - pmf -> quantized CDF ............ DCVC-DC/src/cpp/ops/ops.cpp:24-82
 *   - symbol -> rANS steps + bypass ... DCVC-DC/src/cpp/rans/rans.cpp:76-139
 *   - reverse flush ................... DCVC-DC/src/cpp/rans/rans.cpp:141-168
 *   - decode + bypass decode .......... DCVC-DC/src/cpp/rans/rans.cpp:272-331
 *   - multi-part split + header ....... DCVC-DC/src/cpp/py_rans/py_rans.cpp:22-225
 *   - HEM headerless int32 variant .... DCVC-HEM/src/cpp/rans/rans_interface.cpp:85-244
 * The rANS64 primitives (Rans64EncPut/EncFlush/DecInit/DecGet/DecAdvance) come
 * from the third-party ryg_rans header `rans64.h` pinned at git
 * c9d162d996fd600315af9ae8eb89d832576cb32d
 * (DCVC-DC/src/cpp/3rdparty/ryg_rans/CMakeLists.txt.in:7-9).  That header is
 * NOT vendored in /root/reference, so its published algorithm is restated
 * here (64-bit state, L = 2^31, 32-bit output words written downwards,
 * x' = (x / f) << n + x % f + start, flush = two words low then high).
 * Parity of the rANS64 byte layout is therefore "parity unpinned" against the
 * reference binary; see DESIGN.md (oracle section).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PREC 16
#define RANS_L (1ull << 31)
#define BYP_BITS 4
#define BYP_MAX 15

/* ---------------------------------------------------------------- ops.cpp */
int oracle_pmf_to_quantized_cdf(const float *pmf, int n, int precision,
                                uint32_t *cdf) {
  int i, j;
  uint32_t total = 0;
  cdf[0] = 0;
  for (i = 0; i < n; i++) {
    double r = (double)roundf(pmf[i] * (float)(1 << precision)) + 0.5;
    cdf[i + 1] = (uint32_t)(int64_t)r;
  }
  for (i = 0; i <= n; i++) total += cdf[i];
  if (total == 0) return -1;
  for (i = 0; i <= n; i++)
    cdf[i] = (uint32_t)(((uint64_t)1 << precision) * (uint64_t)cdf[i] / total);
  for (i = 1; i <= n; i++) cdf[i] += cdf[i - 1];
  cdf[n] = 1u << precision;
  for (i = 0; i < n; i++) {
    if (cdf[i] == cdf[i + 1]) {
      uint32_t best_freq = 0xffffffffu;
      int best = -1;
      for (j = 0; j < n; j++) {
        uint32_t f = cdf[j + 1] - cdf[j];
        if (f > 1 && f < best_freq) {
          best_freq = f;
          best = j;
        }
      }
      if (best < 0) return -1;
      if (best < i) {
        for (j = best + 1; j <= i; j++) cdf[j]--;
      } else {
        for (j = i + 1; j <= best; j++) cdf[j]++;
      }
    }
  }
  return 0;
}

/* ------------------------------------------------------------- step list */
typedef struct {
  uint16_t start, range;
  int bypass;
} step_t;

typedef struct {
  step_t *v;
  int64_t n, cap;
} steps_t;

static void push(steps_t *s, uint16_t start, uint16_t range, int bypass) {
  if (s->n == s->cap) {
    s->cap = s->cap ? s->cap * 2 : 1024;
    s->v = (step_t *)realloc(s->v, (size_t)s->cap * sizeof(step_t));
  }
  s->v[s->n].start = start;
  s->v[s->n].range = range;
  s->v[s->n].bypass = bypass;
  s->n++;
}

/* one symbol (rans.cpp:94-136) */
static void add_symbol(steps_t *s, int32_t sym, int idx, const int32_t *cdfs,
                       int stride, const int32_t *sizes,
                       const int32_t *offsets) {
  const int32_t *cdf = cdfs + (int64_t)idx * stride;
  int32_t max_value = sizes[idx] - 2;
  int32_t value = sym - offsets[idx];
  uint32_t raw_val = 0;
  int32_t n_bypass, val, j;
  if (value < 0) {
    raw_val = (uint32_t)(-2 * value - 1);
    value = max_value;
  } else if (value >= max_value) {
    raw_val = (uint32_t)(2 * (value - max_value));
    value = max_value;
  }
  push(s, (uint16_t)cdf[value], (uint16_t)(cdf[value + 1] - cdf[value]), 0);
  if (value == max_value) {
    n_bypass = 0;
    while ((raw_val >> (n_bypass * BYP_BITS)) != 0) n_bypass++;
    val = n_bypass;
    while (val >= BYP_MAX) {
      push(s, BYP_MAX, BYP_MAX + 1, 1);
      val -= BYP_MAX;
    }
    push(s, (uint16_t)val, (uint16_t)(val + 1), 1);
    for (j = 0; j < n_bypass; j++) {
      int32_t v1 = (int32_t)((raw_val >> (j * BYP_BITS)) & BYP_MAX);
      push(s, (uint16_t)v1, (uint16_t)(v1 + 1), 1);
    }
  }
}

/* rans64 restated: Rans64EncPut / Rans64EncPutBits / Rans64EncFlush */
static int64_t flush_steps(const steps_t *s, uint8_t *out) {
  uint32_t *buf = (uint32_t *)malloc((size_t)(s->n + 2) * 4);
  uint32_t *end = buf + s->n + 2, *ptr = end;
  uint64_t x = RANS_L;
  int64_t i, nbytes;
  for (i = s->n - 1; i >= 0; i--) {
    const step_t *st = &s->v[i];
    if (!st->bypass) {
      uint64_t x_max = ((RANS_L >> PREC) << 32) * st->range;
      if (x >= x_max) {
        *--ptr = (uint32_t)x;
        x >>= 32;
      }
      x = ((x / st->range) << PREC) + (x % st->range) + st->start;
    } else {
      uint64_t freq = 1u << (16 - BYP_BITS);
      uint64_t x_max = ((RANS_L >> 16) << 32) * freq;
      if (x >= x_max) {
        *--ptr = (uint32_t)x;
        x >>= 32;
      }
      x = (x << BYP_BITS) | st->start;
    }
  }
  ptr -= 2;
  ptr[0] = (uint32_t)(x >> 0);
  ptr[1] = (uint32_t)(x >> 32);
  nbytes = (int64_t)(end - ptr) * 4;
  if (out) memcpy(out, ptr, (size_t)nbytes);
  free(buf);
  return nbytes;
}

/*
 * DC encoder: `ncalls` encode_with_indexes calls, call c has call_len[c]
 * symbols (concatenated in sym/idx).  Each call is split over `parts` parts
 * (py_rans.cpp:51-65).  Writes the DC stream with header (py_rans.cpp:74-119)
 * into out (capacity cap); returns its size or -1.
 */
int64_t oracle_dc_encode(int ncalls, const int64_t *call_len,
                         const int16_t *sym, const int16_t *idx,
                         const int32_t *cdfs, int stride,
                         const int32_t *sizes, const int32_t *offsets,
                         int parts, uint8_t *out, int64_t cap) {
  steps_t st[16];
  uint8_t *pbuf[16];
  int64_t plen[16];
  int64_t base = 0, total = 0, maxsz = 0, off;
  int c, p, k, per, overhead;
  if (parts < 1 || parts > 16) return -1;
  memset(st, 0, sizeof(st));
  for (c = 0; c < ncalls; c++) {
    int64_t n = call_len[c], each = n / parts;
    for (p = 0; p < parts; p++) {
      int64_t o = p * each, cnt = p < parts - 1 ? each : n - each * (parts - 1);
      int64_t i;
      for (i = 0; i < cnt; i++) {
        int ix = idx[base + o + i];
        if (ix < 0) continue;
        add_symbol(&st[p], sym[base + o + i], ix, cdfs, stride, sizes, offsets);
      }
    }
    base += n;
  }
  for (p = 0; p < parts; p++) {
    plen[p] = flush_steps(&st[p], NULL);
    pbuf[p] = (uint8_t *)malloc((size_t)plen[p]);
    flush_steps(&st[p], pbuf[p]);
    free(st[p].v);
    total += plen[p];
    if (p < parts - 1 && plen[p] > maxsz) maxsz = plen[p];
  }
  per = maxsz > 65535 ? 4 : 2;
  overhead = 1 + (parts > 1 ? (parts - 1) * per : 0);
  if (total + overhead > cap) {
    for (p = 0; p < parts; p++) free(pbuf[p]);
    return -1;
  }
  out[0] = (uint8_t)(((parts - 1) << 4) + (per == 2 ? 1 : 0));
  for (p = 0; p < parts - 1; p++)
    for (k = 0; k < per; k++) out[1 + per * p + k] = (uint8_t)(plen[p] >> (8 * k));
  off = overhead;
  for (p = 0; p < parts; p++) {
    memcpy(out + off, pbuf[p], (size_t)plen[p]);
    off += plen[p];
    free(pbuf[p]);
  }
  return off;
}

/* HEM encoder: int32, single headerless stream (rans_interface.cpp:85-172). */
int64_t oracle_hem_encode(int64_t n, const int32_t *sym, const int32_t *idx,
                          const int32_t *cdfs, int stride, const int32_t *sizes,
                          const int32_t *offsets, uint8_t *out, int64_t cap) {
  steps_t st;
  int64_t i, len;
  memset(&st, 0, sizeof(st));
  for (i = 0; i < n; i++)
    add_symbol(&st, sym[i], idx[i], cdfs, stride, sizes, offsets);
  len = flush_steps(&st, NULL);
  if (len > cap) {
    free(st.v);
    return -1;
  }
  flush_steps(&st, out);
  free(st.v);
  return len;
}

/* ---------------------------------------------------------------- decode */
typedef struct {
  const uint32_t *ptr, *end;
  uint64_t x;
} dstate_t;

static uint32_t rd(dstate_t *d) { return d->ptr < d->end ? *d->ptr++ : 0; }

static int32_t decode_one(dstate_t *d, int ix, const int32_t *cdfs, int stride,
                          const int32_t *sizes, const int32_t *offsets) {
  const int32_t *cdf = cdfs + (int64_t)ix * stride;
  int32_t max_value = sizes[ix] - 2, value, s;
  uint32_t cum = (uint32_t)(d->x & ((1u << PREC) - 1));
  uint64_t start, freq;
  /* linear search as in rans.cpp:295-298 */
  s = 0;
  while (s < sizes[ix] && (uint32_t)cdf[s] <= cum) s++;
  s -= 1;
  start = (uint32_t)cdf[s];
  freq = (uint32_t)(cdf[s + 1] - cdf[s]);
  d->x = freq * (d->x >> PREC) + (d->x & ((1u << PREC) - 1)) - start;
  if (d->x < RANS_L) d->x = (d->x << 32) | rd(d);
  value = s;
  if (value == max_value) {
    int32_t val, n_bypass, raw_val = 0, j;
#define GETBITS(dst)                                     \
  do {                                                   \
    dst = (int32_t)(d->x & BYP_MAX);                     \
    d->x >>= BYP_BITS;                                   \
    if (d->x < RANS_L) d->x = (d->x << 32) | rd(d);      \
  } while (0)
    GETBITS(val);
    n_bypass = val;
    while (val == BYP_MAX) {
      GETBITS(val);
      n_bypass += val;
    }
    for (j = 0; j < n_bypass && j < 8; j++) {
      GETBITS(val);
      raw_val |= val << (j * BYP_BITS);
    }
#undef GETBITS
    value = raw_val >> 1;
    if (raw_val & 1)
      value = -value - 1;
    else
      value += max_value;
  }
  return value + offsets[ix];
}

int oracle_dc_decode(const uint8_t *stream, int64_t len, int ncalls,
                     const int64_t *call_len, const int16_t *idx,
                     const int32_t *cdfs, int stride, const int32_t *sizes,
                     const int32_t *offsets, int parts, int16_t *out) {
  dstate_t d[16];
  uint32_t *words[16];
  int64_t sizes_b[16], off = 1, tot = 0, base = 0;
  int flag = stream[0], nstreams = (flag >> 4) + 1;
  int per = (flag & 0x0f) == 1 ? 2 : 4, p, c, k;
  if (nstreams != parts) return -1;
  for (p = 0; p < nstreams - 1; p++) {
    int64_t s = 0;
    for (k = 0; k < per; k++) s |= (int64_t)stream[off + k] << (8 * k);
    off += per;
    sizes_b[p] = s;
    tot += s;
  }
  sizes_b[nstreams - 1] = len - off - tot;
  for (p = 0; p < nstreams; p++) {
    words[p] = (uint32_t *)malloc((size_t)sizes_b[p] + 8);
    memcpy(words[p], stream + off, (size_t)sizes_b[p]);
    off += sizes_b[p];
    d[p].ptr = words[p];
    d[p].end = words[p] + sizes_b[p] / 4;
    d[p].x = (uint64_t)rd(&d[p]);
    d[p].x |= (uint64_t)rd(&d[p]) << 32;
  }
  for (c = 0; c < ncalls; c++) {
    int64_t n = call_len[c], each = n / parts, i;
    for (p = 0; p < parts; p++) {
      int64_t o = p * each, cnt = p < parts - 1 ? each : n - each * (parts - 1);
      for (i = 0; i < cnt; i++) {
        int ix = idx[base + o + i];
        if (ix < 0) {
          out[base + o + i] = 0;
          continue;
        }
        out[base + o + i] =
            (int16_t)decode_one(&d[p], ix, cdfs, stride, sizes, offsets);
      }
    }
    base += n;
  }
  for (p = 0; p < nstreams; p++) free(words[p]);
  return 0;
}

int oracle_hem_decode(const uint8_t *stream, int64_t len, int64_t n,
                      const int32_t *idx, const int32_t *cdfs, int stride,
                      const int32_t *sizes, const int32_t *offsets,
                      int32_t *out) {
  dstate_t d;
  int64_t i;
  uint32_t *w = (uint32_t *)malloc((size_t)len + 8);
  memcpy(w, stream, (size_t)len);
  d.ptr = w;
  d.end = w + len / 4;
  d.x = (uint64_t)rd(&d);
  d.x |= (uint64_t)rd(&d) << 32;
  for (i = 0; i < n; i++)
    out[i] = decode_one(&d, idx[i], cdfs, stride, sizes, offsets);
  free(w);
  return 0;
}
