/*
 * dcvc_rans.h — C ABI of the host entropy coder (libdcvc_rans.so).
 *
 * This is the drop-in replacement for the reference's pybind11 coder modules.
 * Every entry point below names the reference interface it replaces.  Plain
 * C types only: pointers + sizes + int status codes, no Python or torch types.
 *
 * Two stream formats are produced, matching the two reference coders:
 *   - DC  format (DCVC-DC, `MLCodec_rans.RansEncoder/RansDecoder`):
 *       int16 symbols/indexes, negative index = "skip" symbol, optional
 *       multi-part streams with a leading flag byte and per-part sizes
 *       (DCVC-DC/src/cpp/py_rans/py_rans.cpp:74-119, 133-164).
 *   - HEM format (DCVC-HEM, `MLCodec_rans.BufferedRansEncoder/RansDecoder`):
 *       int32 symbols/indexes, a single headerless stream
 *       (DCVC-HEM/src/cpp/rans/rans_interface.cpp:85-244).
 * Both share the rANS64 core (64-bit state, 32-bit renormalisation words,
 * 16-bit probability precision) with 4-bit bypass escape coding
 * (DCVC-DC/src/cpp/rans/rans.cpp:37-168, 272-331).
 */
#ifndef DCVC_RANS_H
#define DCVC_RANS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes */
#define DCVC_OK 0
#define DCVC_EINVAL (-1)  /* bad argument / bad index / null pointer     */
#define DCVC_ERANGE (-2)  /* symbol too far from its offset to escape-code */
#define DCVC_ENOMEM (-3)
#define DCVC_ESTREAM (-4) /* malformed or truncated stream               */
#define DCVC_EBUSY (-5)   /* stream requested before flush()            */

/* Replaces MLCodec_CXX.pmf_to_quantized_cdf (DCVC-DC/src/cpp/ops/ops.cpp:24-82,
 * identical in DCVC-HEM).  `pmf` has n entries, `cdf_out` receives n+1. */
int dcvc_pmf_to_quantized_cdf(const float *pmf, int n, int precision,
                              uint32_t *cdf_out);

/* ---- CDF tables ---------------------------------------------------------
 * The reference copies the whole [cdf_num, cdf_stride] int32 table into
 * std::vectors on every encode/decode call (py_rans.cpp:36-49).  Here a table
 * is uploaded once and referenced by handle; it also carries the decoder's
 * symbol lookup accelerator.  The layout is the reference's own:
 * cdfs[i*cdf_stride + j], cdf_sizes[i] valid entries, offsets[i]. */
typedef struct dcvc_cdf_table dcvc_cdf_table;
dcvc_cdf_table *dcvc_cdf_table_create(const int32_t *cdfs, int cdf_num,
                                      int cdf_stride, const int32_t *cdf_sizes,
                                      const int32_t *offsets);
void dcvc_cdf_table_destroy(dcvc_cdf_table *t);

/* ---- encoder -------------------------------------------------------------
 * Replaces RansEncoder(bool multiThread, int streamPart)
 * (DCVC-DC/src/cpp/py_rans/py_rans.cpp:11-20) and, with stream_part = 1 and
 * no header, BufferedRansEncoder() (DCVC-HEM rans_interface.hpp:49).
 * multithread != 0 runs symbol buffering + flush on a worker thread per part
 * (RansEncoderLibMultiThread, DCVC-DC/src/cpp/rans/rans.cpp:174-263);
 * calls then return immediately and get_stream() blocks for the result. */
typedef struct dcvc_rans_enc dcvc_rans_enc;
dcvc_rans_enc *dcvc_rans_enc_create(int multithread, int stream_part);
void dcvc_rans_enc_destroy(dcvc_rans_enc *e);

/* Replaces RansEncoder::encode_with_indexes (py_rans.cpp:22-66) with the
 * reference's argument list.  Symbols are split into stream_part equal
 * slices, the last slice taking the remainder. */
int dcvc_rans_enc_encode_with_indexes_i16(dcvc_rans_enc *e,
                                          const int16_t *symbols,
                                          const int16_t *indexes, int64_t n,
                                          const int32_t *cdfs, int cdf_num,
                                          int cdf_stride,
                                          const int32_t *cdf_sizes,
                                          const int32_t *offsets);
/* Same, with a pre-uploaded table. */
int dcvc_rans_enc_encode_table_i16(dcvc_rans_enc *e, const int16_t *symbols,
                                   const int16_t *indexes, int64_t n,
                                   const dcvc_cdf_table *t);
/* Replaces BufferedRansEncoder::encode_with_indexes (HEM, int32; a symbol
 * whose |value - offset| >= 2^27 is rejected with DCVC_ERANGE instead of the
 * reference's non-terminating bypass loop, rans_interface.cpp:122-125). */
int dcvc_rans_enc_encode_table_i32(dcvc_rans_enc *e, const int32_t *symbols,
                                   const int32_t *indexes, int64_t n,
                                   const dcvc_cdf_table *t);

/* Replaces RansEncoder::flush (py_rans.cpp:68-72 / rans.cpp:141-168). */
int dcvc_rans_enc_flush(dcvc_rans_enc *e);
/* Size in bytes of the flushed stream; with_header = 1 gives the DC format
 * (flag byte + part sizes, py_rans.cpp:74-119), 0 the raw HEM format
 * (only valid for stream_part == 1).  Blocks until flush has completed. */
int64_t dcvc_rans_enc_stream_size(dcvc_rans_enc *e, int with_header);
/* Replaces RansEncoder::get_encoded_stream / BufferedRansEncoder::flush's
 * return value.  Writes at most cap bytes, returns bytes written or <0. */
int64_t dcvc_rans_enc_get_stream(dcvc_rans_enc *e, int with_header,
                                 uint8_t *out, int64_t cap);
/* Replaces RansEncoder::reset (py_rans.cpp:121-125). */
int dcvc_rans_enc_reset(dcvc_rans_enc *e);

/* ---- decoder -------------------------------------------------------------
 * Replaces RansDecoder(int streamPart) (py_rans.cpp:127-131) and HEM
 * RansDecoder() (rans_interface.cpp:176-244). */
typedef struct dcvc_rans_dec dcvc_rans_dec;
dcvc_rans_dec *dcvc_rans_dec_create(int stream_part);
void dcvc_rans_dec_destroy(dcvc_rans_dec *d);
/* Replaces RansDecoder::set_stream (py_rans.cpp:133-164 with_header = 1;
 * rans_interface.cpp:176-182 with_header = 0).  The bytes are copied. */
int dcvc_rans_dec_set_stream(dcvc_rans_dec *d, const uint8_t *data,
                             int64_t len, int with_header);
/* Replaces RansDecoder::decode_stream (py_rans.cpp:166-225, parts decoded in
 * parallel threads like the reference's std::async). */
int dcvc_rans_dec_decode_with_indexes_i16(dcvc_rans_dec *d,
                                          const int16_t *indexes, int64_t n,
                                          const int32_t *cdfs, int cdf_num,
                                          int cdf_stride,
                                          const int32_t *cdf_sizes,
                                          const int32_t *offsets,
                                          int16_t *out);
int dcvc_rans_dec_decode_table_i16(dcvc_rans_dec *d, const int16_t *indexes,
                                   int64_t n, const dcvc_cdf_table *t,
                                   int16_t *out);
int dcvc_rans_dec_decode_table_i32(dcvc_rans_dec *d, const int32_t *indexes,
                                   int64_t n, const dcvc_cdf_table *t,
                                   int32_t *out);

/* ---- threads ---------------------------------------------------------------
 * Every encoder and decoder of the process works its stream parts on one
 * shared pool of persistent worker threads (plus the calling thread), not on
 * threads of its own (the reference's RansEncoderLibMultiThread keeps one
 * worker per encoder, rans.h:83-109, and RansDecoder starts one std::async
 * per part per call, py_rans.cpp:197-211).  dcvc_rans_set_threads(n) fixes
 * the worker count before the first coder is created (default: the
 * DCVC_CODER_THREADS environment variable, else min(15, hardware threads - 1));
 * afterwards it returns DCVC_EBUSY unless n is the running count.
 * dcvc_rans_threads() starts the pool if needed and returns its workers. */
int dcvc_rans_set_threads(int workers);
int dcvc_rans_threads(void);

#ifdef __cplusplus
}
#endif
#endif /* DCVC_RANS_H */
