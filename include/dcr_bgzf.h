/* dcr_bgzf.h — native BGZF stream codec for the host side of the drop-in.
 *
 * The reference reads and writes BAM through pysam/htslib
 * (DuplexUMIConsensusReads.py:1476 AlignmentFile(input, "rb"),
 *  :1494-1502 AlignmentFile(..., "wb", template=inbam), :1519 iteration,
 *  :1526/:1551/:1594 write, :1646-1649 close).  pysam is absent from this
 * image; duplexumiconsensusreads_amd/bam.py keeps the BAM record layout in
 * Python and takes its byte stream from these functions (SURVEY.md §8f ranks
 * 1 and 2: the BGZF inflate/deflate that bound whole-file throughput).
 *
 * Blocks are inflated / deflated on a pool of host threads, a batch of blocks
 * at a time, and consumed / written in file order.  Output is byte-identical
 * to zlib deflate(level, raw, memLevel 8) over 0xff00-byte blocks, i.e. the
 * same file bam.BGZFWriter produces.  Not thread-safe per handle.
 */
#ifndef DCR_BGZF_H
#define DCR_BGZF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dcr_bgzf_reader dcr_bgzf_reader;
typedef struct dcr_bgzf_writer dcr_bgzf_writer;

/* Open a BGZF file for reading; n_threads <= 0 picks the host's core count
 * (capped at 16).  NULL on error (message in dcr_bgzf_last_error()). */
dcr_bgzf_reader* dcr_bgzf_open_read(const char* path, int n_threads);

/* Copy up to n decompressed bytes into dst.  Returns the count (< n only at
 * end of file), or -1 on a format / CRC / I/O error. */
int64_t dcr_bgzf_read(dcr_bgzf_reader* r, void* dst, int64_t n);

void dcr_bgzf_close_read(dcr_bgzf_reader* r);

/* Open a BGZF file for writing at zlib level `level` (bam.py uses 6). */
dcr_bgzf_writer* dcr_bgzf_open_write(const char* path, int level, int n_threads);

/* Append n bytes; returns 0, or -1 on error. */
int dcr_bgzf_write(dcr_bgzf_writer* w, const void* src, int64_t n);

/* Flush the partial block, append the BGZF EOF marker, close.  0 or -1. */
int dcr_bgzf_close_write(dcr_bgzf_writer* w);

/* Index complete BAM records ("<i block_size> + body") in buf[0, n): writes
 * the byte offset of each record's block_size field into offs (at most
 * max_recs) and the bytes spanned by complete records into *consumed.
 * Returns the record count, or -1 on a negative block_size. */
int64_t dcr_bam_index_records(const uint8_t* buf, int64_t n, int64_t* offs, int64_t max_recs,
                              int64_t* consumed);

/* Thread-local message of the last failure. */
const char* dcr_bgzf_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* DCR_BGZF_H */
