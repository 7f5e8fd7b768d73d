/*
 * dcr_io.h — C-ABI of the native host side around the consensus kernels
 * (libdcr_io.so, built with g++; no GPU code).
 *
 * The reference does its I/O and per-family bookkeeping in Python over pysam
 * (/root/reference/DuplexUMIConsensusReads.py, cited as :line):
 *
 *   ingest  (dcr_ingest_*)  replaces the streaming loop's front half
 *       for read in inbam                       :1519
 *       pass_filters                            :1135-1181  (+ excluded-reads side file :1523-1528)
 *       add_read_to_family / load_next_family   :1185-1217, :329-342
 *       preprocess_family up to the read loop   :1248-1264
 *           check_family_UMIs / check_family_rnames :100-128
 *           split_family                        :132-154
 *           check_number_reads (random.sample)  :157-188  (CPython MT19937, state in/out)
 *       filtered-families side file             :1546-1555, :1611-1614
 *     and packs every processed family straight into the dcr_batch layout
 *     (include/dcr.h) the GPU consumes, in caller-owned (pinned) memory.
 *
 *   writer  (dcr_fmt_*)     replaces the record half of the loop's back end
 *       make_consensus_read record build        :1352-1384
 *       get_consensus_id / get_consensus_flag   :892-968
 *       add_tags (method="double_strand")       :1076-1120
 *       fix_paired_end_fields                   :1390-1419
 *       consensusbam.write                      :1593-1594
 *     formatting the two duplex records per family from kernel outputs.
 *
 *   BGZF (dcr_bgzf_*, include/dcr_bgzf.h) is the byte stream under both.
 *
 * Errors: functions return 0 / a DCR_IO_E* code, message from
 * dcr_io_last_error() (thread-local).  "The reference would exit / raise
 * here" is not an error of the call: it is reported in the batch (end_kind).
 */
#ifndef DCR_IO_H
#define DCR_IO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCR_IO_ABI_VERSION 1

enum { DCR_IO_OK = 0, DCR_IO_EARG = 1, DCR_IO_EFILE = 2, DCR_IO_EFORMAT = 3, DCR_IO_ECAPACITY = 4 };

/* batch end kinds */
enum {
    DCR_END_FULL = 0,   /* a capacity was reached; more input follows          */
    DCR_END_EOF = 1,    /* input exhausted; the last family is in this batch   */
    DCR_END_ERROR = 2   /* the reference stops here (err_kind, err_msg)        */
};

/* what the reference does at the batch's error point */
enum {
    DCR_ERR_NONE = 0,
    DCR_ERR_EXIT = 1,        /* print(err_msg); sys.exit(1)                       */
    DCR_ERR_TYPE = 2,        /* TypeError                                         */
    DCR_ERR_INDEX = 3,       /* IndexError                                        */
    DCR_ERR_VALUE = 4,       /* ValueError                                        */
    DCR_ERR_ATTRIBUTE = 5    /* AttributeError (a non-string MI / RX tag)         */
};

/* family table kinds */
enum { DCR_FAM_PROCESSED = 0, DCR_FAM_FILTERED = 1 };

typedef struct dcr_ingest_cfg {
    int32_t min_map_quality;   /* -q (mapQ_threshold)                            */
    int32_t min_reads;         /* --min_reads                                    */
    int32_t max_reads;         /* --max_reads                                    */
    int32_t min_base_quality;  /* --min_base_quality (=/X count after the trim)  */
    int32_t n_threads;         /* inflate / pack threads (0: up to 16)           */
    int32_t flags;             /* DCR_INGEST_* below (0: defaults)               */
} dcr_ingest_cfg;

/* dcr_ingest_cfg.flags: inflate on the host pool even when a GPU inflate
 * hook is set (dcr_io_set_inflate_hook), e.g. a count-only pass running
 * beside a GPU pass */
#define DCR_INGEST_HOST_INFLATE 1

/* One host batch.  The caller allocates every array (pinned memory for the
 * GPU path) and sets the capacities; dcr_ingest_next fills it.  The first
 * twelve arrays are exactly a dcr_batch (include/dcr.h) over the processed
 * families.  Family table entries cover every family completed in the batch
 * (processed and filtered), in input order. */
typedef struct dcr_host_batch {
    /* capacities (caller) */
    int32_t cap_fam;        /* processed families                        */
    int32_t cap_tab;        /* family table entries                      */
    int32_t cap_reads;
    int32_t reserved0;
    int64_t cap_cigar;
    int64_t cap_bases;
    int64_t cap_names;      /* bytes of the string arena                 */
    int64_t cap_side;       /* bytes of each side-record buffer          */
    /* dcr_batch arrays */
    int32_t *sub_off;       /* [4*cap_fam+1] */
    int32_t *read_pos;
    uint8_t *read_mapq;
    int64_t *seq_off;
    int32_t *seq_len;
    int32_t *cig_off;
    int32_t *cig_n;
    uint32_t *cigar;
    uint8_t *bases;
    uint8_t *quals;
    int64_t *ss_col_off;    /* [4*cap_fam+1] */
    int64_t *ds_col_off;    /* [2*cap_fam+1] */
    /* per processed family (writer metadata) */
    int32_t *fam_tid;       /* [cap_fam] reference_id of the family          */
    int64_t *fam_code;      /* [cap_fam] names offset of the family code (MI prefix) */
    int64_t *fam_rx;        /* [2*cap_fam] names offsets: RX of A1 read0, of B1 read0 */
    uint16_t *fam_eqx;      /* [4*cap_fam] reads whose CIGAR still holds =/X after the trim (:374-375) */
    /* family table */
    int32_t *tab_kind;      /* [cap_tab] DCR_FAM_*                            */
    int32_t *tab_proc;      /* [cap_tab] processed index, or -1               */
    int32_t *tab_sampled;   /* [cap_tab] bit k: subfamily k was downsampled   */
    int64_t *tab_code;      /* [cap_tab] names offset of the family code      */
    int64_t *tab_exc_cut;   /* [cap_tab] excluded-reads bytes written before the family is processed */
    int64_t *tab_filt_cut;  /* [cap_tab] filtered-families bytes written before it */
    char *names;            /* NUL-terminated strings                        */
    uint8_t *side_exc;      /* raw BAM records (block_size + body) for _filteredreads.bam    */
    uint8_t *side_filt;     /* raw BAM records for _filteredfamilies.bam                     */
    /* filled by dcr_ingest_next */
    int32_t n_fam, n_reads;
    int64_t n_cigar, n_bases, ss_cols, ds_cols;
    int32_t n_tab, end_kind;
    int64_t n_names, n_side_exc, n_side_filt;
    int32_t err_kind, reserved1;
    char err_msg[512];
} dcr_host_batch;

typedef struct dcr_ingest dcr_ingest;

int dcr_io_abi_version(void);
const char *dcr_io_last_error(void);

/* open a BAM; NULL on failure (unreadable or not a BGZF/BAM file) */
dcr_ingest *dcr_ingest_open(const char *path, const dcr_ingest_cfg *cfg);
void dcr_ingest_close(dcr_ingest *ing);
/* the header as stored (magic "BAM\1" .. references), for the output files */
int64_t dcr_ingest_header(dcr_ingest *ing, const uint8_t **bytes);
/* CPython random.Random state (getstate()[1]: 624 words + index) in / out */
int dcr_ingest_set_rng(dcr_ingest *ing, const uint32_t *mt624, int32_t index);
int dcr_ingest_get_rng(dcr_ingest *ing, uint32_t *mt624, int32_t *index);
/* fill the next batch; 0 on success (see hb->end_kind) */
int dcr_ingest_next(dcr_ingest *ing, dcr_host_batch *hb);
/* counters so far: [0] passed reads, [1] excluded reads, [2] processed
   families, [3] filtered families, [4] records read */
int dcr_ingest_counters(dcr_ingest *ing, int64_t *out5);

/* ---- BGZF inflate on the GPU (include/dcr_inflate.h) ----------------------
 * With a hook set, ingests opened afterwards hand the BGZF members of every
 * input chunk to hook->run (libdcr.so's device inflater: the members' CRC32
 * and ISIZE are checked there) instead of inflating them on the host pool,
 * and take their chunk buffers from hook->host_alloc (page-locked).  NULL
 * clears it.  DCR_GPU_INFLATE=0 in the environment ignores a set hook (A/B
 * runs).  The struct is copied; its functions must outlive the ingests. */
struct dcr_inflate_hook;
int dcr_io_set_inflate_hook(const struct dcr_inflate_hook *hook);
/* 1 if the ingest inflates on the GPU */
int dcr_ingest_gpu_inflate(dcr_ingest *ing);

/* ---- family-range sharding (cli --gpus N: one process per GPU) ----------
 * Split points for n_parts ranges of whole families: part p (p >= 1) starts
 * at voff[p-1], the BGZF virtual offset (block file offset << 16 | offset in
 * the block's data) of a passing read whose MI code differs from that of the
 * passing read before it: a family start in the reference's grouping
 * (:1185-1217), found near p/n of the file.  A record boundary near the
 * target is found by checking a run of consecutive records field by field;
 * the rank before checks that its own record chain arrives exactly there.
 * -1 where no point was found near the target (the part is then empty).
 * Returns 0 or an error code (dcr_io_last_error). */
int dcr_split_points(const char *path, int32_t n_parts, const dcr_ingest_cfg *cfg, int64_t *voff);
/* open the records of [start_voff, end_voff): start 0 = the file start
 * (header parsed), end -1 = the end of the file.  A range that stops before
 * the end of the file completes its last family at the range end, as the
 * reference does when the next family's first read arrives. */
dcr_ingest *dcr_ingest_open_range(const char *path, const dcr_ingest_cfg *cfg, int64_t start_voff, int64_t end_voff);
/* the (population, sample size) pair of every random.sample call so far, in
 * order (check_number_reads :157-188): returns the count, copies up to cap
 * pairs into out */
int64_t dcr_ingest_sample_calls(dcr_ingest *ing, int32_t *out, int64_t cap);
/* State gate of a range that starts after other ranges (the sharded CLI):
 * called once, on the thread running dcr_ingest_next, right before the
 * range's first random.sample call, it writes the exact generator state to
 * sample from (the state after every earlier range's calls) and returns 0;
 * a range that never samples never calls it.  Nonzero ends the ingest with
 * an error.  NULL removes the gate. */
typedef int (*dcr_state_gate_fn)(void *user, uint32_t *mt624, int32_t *index);
int dcr_ingest_set_state_gate(dcr_ingest *ing, dcr_state_gate_fn fn, void *user);
/* random.sample(range(n_i), k_i) for each pair: the state after those calls */
int dcr_py_replay(uint32_t *mt624, int32_t *index, const int32_t *calls, int64_t n_calls);
/* the BAM header as stored (magic .. references) without opening an ingest:
 * returns its length (copied when <= cap), or -1 */
int64_t dcr_bam_header(const char *path, uint8_t *out, int64_t cap);

/* CPython random.sample(range(n), k) on the given state (tests) */
int dcr_py_sample(uint32_t *mt624, int32_t *index, int32_t n, int32_t k, int32_t *out);

/* ---- BGZF writer (libdeflate, blocks of 0xff00 bytes deflated on a pool) ---- */
typedef struct dcr_bgzw dcr_bgzw;
/* level 0..12 (libdeflate levels; htslib's default is 6) */
dcr_bgzw *dcr_bgzw_open(const char *path, int level, int n_threads);
int dcr_bgzw_write(dcr_bgzw *w, const void *bytes, int64_t n);
/* append already compressed BGZF blocks (n bytes, holding raw_bytes of
   data), after flushing what write() left pending */
int dcr_bgzw_put_blocks(dcr_bgzw *w, const void *blocks, int64_t n, int64_t raw_bytes);
/* flush, write the BGZF EOF marker, close; 0 on success */
int dcr_bgzw_close(dcr_bgzw *w);
/* bytes written so far (compressed, uncompressed) */
int dcr_bgzw_sizes(dcr_bgzw *w, int64_t *out2);

/* ---- consensus records ----
 * Host copies of the kernel outputs the records need (include/dcr.h
 * dcr_out): single-strand status, mapq, len, n_de, D, M, E, seq, qual, d, e;
 * duplex: every field.  Regions follow hb->ss_col_off / hb->ds_col_off. */
typedef struct dcr_fmt_out {
    const uint8_t *status;
    const int32_t *pos, *mapq, *len, *n_cig, *n_de, *D, *M;
    const double *E;
    const uint8_t *seq, *qual;
    const uint32_t *cigar;
    const uint16_t *d, *e;
} dcr_fmt_out;

/* what the reference raises for a processed family, in its execution order */
enum {
    DCR_FAIL_NONE = 0,
    DCR_FAIL_INDEX = 1, DCR_FAIL_TYPE = 2, DCR_FAIL_VALUE = 3, DCR_FAIL_OVERFLOW = 4,
    DCR_FAIL_EXIT_BADCHAR = 5,
    DCR_FAIL_UNICODE = 7   /* pysam force_bytes(ascii) of an aq/bq tag: a quality >= 95 */
};

/* First failing processed family in [0, n_fam), or n_fam if none; its
 * DCR_FAIL_* in *kind and where it fails in *which: 0..3 the single-strand
 * consensus of that subfamily, 4..5 the duplex one, 8 + k the preprocessing
 * of a read of subfamily k (single-strand status DCR_ST_PREP | s, include/dcr.h).
 * read_status is unused (kept for the ABI). */
int32_t dcr_fmt_scan(const dcr_host_batch *hb, const dcr_fmt_out *ss, const dcr_fmt_out *ds,
                     const int32_t *read_status, int32_t n_fam, int32_t *kind, int32_t *which);
/* Format the two duplex records of processed families [0, n_fam) (records
 * of families that fail must not be in the range) and write them. */
int dcr_fmt_write(dcr_bgzw *w, const dcr_host_batch *hb, const dcr_fmt_out *ss, const dcr_fmt_out *ds,
                  int32_t n_fam);

/* ---- the GPU BGZF block compressor (csrc/dcr_deflate.h) emulated lane by
 * lane on the host, for tests: one BGZF block of in[0, n) (n <= 0xff00) into
 * out (>= 64 KiB); returns its size or -1 */
int64_t dcr_deflate_emulate(const uint8_t *in, int64_t n, uint8_t *out);
/* (test) codes per length of the device's batched Huffman code-length count
 * (dcr_deflate.h mr_counts) and of the plain in-place algorithm, for freq[0..m)
 * ascending and nonzero, m in 2..288; 0, or -1 on bad arguments */
int dcr_deflate_lengths_ab(const uint32_t *freq, int m, uint32_t *num_a, uint32_t *num_b);

/* ---- synthetic inputs (bench / tests) ----
 * Records of n_fam duplex families from dcr_batch-layout arrays (reads of
 * family f's subfamily k = A1 B2 B1 A2 at sub_off[4f+k] ..), fgbio
 * GroupReadsByUmi style: flags 99 163 83 147, MI "<fam>/A|B", RX "U1-U2" on
 * A and "U2-U1" on B (umis: 16 letters per family), names mol<fam>_<k>_<j>. */
typedef struct dcr_synth_in {
    int32_t n_fam, tid;
    int64_t fam_id0;
    const int32_t *sub_off, *read_pos;
    const uint8_t *read_mapq;
    const int64_t *seq_off;
    const int32_t *seq_len, *cig_off, *cig_n;
    const uint32_t *cigar;
    const uint8_t *bases, *quals;
    const char *umis;
} dcr_synth_in;
int dcr_synth_write(dcr_bgzw *w, const dcr_synth_in *in, int n_threads);

#ifdef __cplusplus
}
#endif
#endif /* DCR_IO_H */
