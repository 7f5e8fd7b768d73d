/*
 * dcr_inflate.h — BGZF inflate on the GPU (libdcr.so) and the hook through
 * which the native BAM ingest (libdcr_io.so, include/dcr_io.h) hands it the
 * blocks of each input chunk instead of inflating them on its host pool.
 *
 * Replaces, for the input side of the reference's loop, pysam's BGZF read
 * under ``for read in samfile.fetch(until_eof=True)``
 * (/root/reference/DuplexUMIConsensusReads.py:1476, :1519): every BGZF member
 * (RFC 1952 gzip member with the "BC" extra field, SAM spec v1.6 §4.1) of a
 * chunk is one raw RFC 1951 stream, inflated by one wavefront
 * (csrc/dcr_inflate.hip); its CRC32 and ISIZE are checked on the device.
 *
 * Plain pointers and sizes only; functions return 0 or a DCR_E* code
 * (include/dcr.h) with the message in dcr_last_error().
 */
#ifndef DCR_INFLATE_H
#define DCR_INFLATE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* one BGZF member of a chunk: its deflate data and where its output goes */
typedef struct dcr_bgzf_member {
    int64_t in_off;     /* first byte of the raw deflate data, from the chunk's compressed base */
    int64_t out_off;    /* first output byte, from the chunk's output base */
    uint32_t in_len;    /* bytes of deflate data (BSIZE - XLEN - 19) */
    uint32_t isize;     /* ISIZE from the member trailer (<= 65536) */
    uint32_t crc;       /* CRC32 from the member trailer */
    uint32_t pad;
} dcr_bgzf_member;

/* The ingest's inflate hook (set with dcr_io_set_inflate_hook, dcr_io.h).
 *   run:        inflate n members: compressed bytes at in[0, in_bytes), output
 *               to out[0, out_bytes); 0 on success, otherwise the index + 1
 *               of the first member that failed (bad stream, ISIZE or CRC32),
 *               or -1 for a runtime error
 *   host_alloc: page-locked host memory for the ingest's chunk buffers and
 *               its compressed staging (NULL: the ingest uses its own)
 *   host_free:  returns such memory */
typedef struct dcr_inflate_hook {
    void *user;
    int (*run)(void *user, const uint8_t *in, int64_t in_bytes, const dcr_bgzf_member *m, int32_t n, uint8_t *out,
               int64_t out_bytes);
    void *(*host_alloc)(void *user, size_t bytes);
    void (*host_free)(void *user, void *p);
    /* streaming (a mapped input): stream_open starts a stream over `file`;
     * stream_add appends members in input order (in_off from `file`, out_off
     * from the first member's output; last != 0 after the final ones), which
     * the device inflates ahead of the reader in large launches on its own
     * thread; stream_fetch blocks until output bytes [out_off, out_off + n)
     * are inflated and copies them to dst (page-locked: a DMA), returning 0,
     * the index + 1 of a failed member, or -1; stream_close stops and frees.
     * NULL stream_open: chunks go through run. */
    void *(*stream_open)(void *user, const uint8_t *file);
    int (*stream_add)(void *stream, const dcr_bgzf_member *m, int32_t n, int32_t last);
    int (*stream_fetch)(void *stream, int64_t out_off, int64_t n, uint8_t *dst);
    void (*stream_close)(void *stream);
} dcr_inflate_hook;

/* libdcr.so: a device inflater (one per process and device; its streams,
 * device buffers and a cache of page-locked host buffers persist across
 * ingests) */
typedef struct dcr_inflater dcr_inflater;
dcr_inflater *dcr_inflater_create(int device);
void dcr_inflater_destroy(dcr_inflater *h);
/* fills *hook with this inflater's run / host_alloc / host_free */
int dcr_inflater_hook(dcr_inflater *h, dcr_inflate_hook *hook);
/* synchronous inflate of n members (host pointers): 0, the index + 1 of the
 * first member that failed (bad stream, ISIZE or CRC32; dcr_last_error names
 * it), or -DCR_E* for bad arguments or a runtime error */
int dcr_inflater_run(dcr_inflater *h, const uint8_t *in, int64_t in_bytes, const dcr_bgzf_member *m, int32_t n,
                     uint8_t *out, int64_t out_bytes);
/* the streaming entry points behind dcr_inflate_hook.stream_* */
typedef struct dcr_inflate_stream dcr_inflate_stream;
dcr_inflate_stream *dcr_inflate_stream_open(dcr_inflater *h, const uint8_t *file);
int dcr_inflate_stream_add(dcr_inflate_stream *st, const dcr_bgzf_member *m, int32_t n, int32_t last);
int dcr_inflate_stream_fetch(dcr_inflate_stream *st, int64_t out_off, int64_t n, uint8_t *dst);
void dcr_inflate_stream_close(dcr_inflate_stream *st);
/* device time of the last run's kernel (ms) and its member count */
int dcr_inflater_last(dcr_inflater *h, float *kernel_ms, int32_t *n_members);
/* totals since creation or the last reset: out4 = {kernel ms, runs, members,
   output bytes}; reset != 0 zeroes them after reading */
int dcr_inflater_totals(dcr_inflater *h, double *out4, int reset);

#ifdef __cplusplus
}
#endif
#endif
