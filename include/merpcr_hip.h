/*
 * merpcr_hip.h -- C ABI of libmerpcr_hip.so, the MI355X (gfx950) STS-search engine.
 *
 * The reference (FOI-Bioinformatics/merpcr) has no FFI layer; its hot path is the
 * Python call chain MerPCR.search -> _process_thread -> _match_sts -> _compare_seqs
 * (src/merpcr/core/engine.py:365-642), fed by the seed table that load_sts_file
 * builds (engine.py:193-329) and by FASTALoader's filtered sequences
 * (src/merpcr/io/fasta.py:18-71).  This header is the seam that replaces that chain:
 * each entry point names the reference routine it stands in for.
 *
 * Conventions: plain pointers and sizes, no C++ or torch types.  Every function
 * returns 0 on success and a negative MP_E* code on failure; mp_last_error()
 * returns a thread-local message for the last failure.  `stream` is a hipStream_t
 * passed as void* (NULL = the legacy default stream).  Handles are opaque and own
 * their device memory; the caller owns every host buffer for the duration of a call.
 */
#ifndef MERPCR_HIP_H
#define MERPCR_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MP_ABI_VERSION 3  /* 2: mp_search_options without fuse_tails; mp_table_layout.
                             3: mp_table_create_ex, mp_search_options form/tuning fields (no
                             environment switches), mp_search_put_hits reports the need,
                             mp_multi_set_gather */

#define MP_OK 0
#define MP_E_ARG (-1)     /* bad argument (maps to ValueError) */
#define MP_E_HIP (-2)     /* HIP runtime / device failure (RuntimeError) */
#define MP_E_NOMEM (-3)   /* device or host allocation failed */
#define MP_E_STATE (-4)   /* handle used out of order (e.g. search before seal) */
#define MP_E_CAP (-5)     /* caller's output buffer too small; *n_hits has the need */
#define MP_E_IO (-6)      /* file cannot be opened or read (OSError) */
#define MP_E_DECODE (-7)  /* input is not valid UTF-8 (UnicodeDecodeError) */

/* Search parameters: the MerPCR constructor arguments that reach the hot path
 * (engine.py:47-97).  Bounds are the reference's (W 3..16, N 0..10, M 0..10000,
 * X >= 0, I 0/1). */
typedef struct mp_params {
    int32_t wordsize;          /* W  (-W) */
    int32_t margin;            /* M  (-M) */
    int32_t mismatches;        /* N  (-N) */
    int32_t three_prime_match; /* X  (-X) */
    int32_t iupac_mode;        /* I  (-I) */
} mp_params;

/* One hit in the reference's output order (engine.py:434-444): 0-based pos1/pos2
 * relative to its sequence, the sequence's index in the genome handle, and the
 * oriented STS record's index in MerPCR.sts_records. */
typedef struct mp_hit {
    uint64_t pos1;
    uint64_t pos2;
    uint32_t seq;
    uint32_t rec;
} mp_hit;

/* Owned range of a search, in (sequence, amplicon start k) order: hits whose
 * (seq, k) is >= (seq_begin, k_begin) and < (seq_end, k_end) are produced.  This is
 * the unit of multi-GPU sharding; {0,0,n_seq,0} is the whole genome. */
typedef struct mp_range {
    uint32_t seq_begin;
    uint32_t seq_end;      /* exclusive; k_end applies inside sequence seq_end */
    uint64_t k_begin;
    uint64_t k_end;
} mp_range;

/* ---- library ------------------------------------------------------------- */
int32_t mp_abi_version(void);
const char* mp_last_error(void);
/* Number of visible HIP devices (0 on a host without a GPU). */
int mp_device_count(int32_t* n);

/* ---- seed table (replaces MerPCR.sts_table / sts_records, engine.py:193-329) --
 * Records are the oriented STS records in sts_records order ('+' then '-' per STS
 * line).  key/hash_off are _hash_value()'s (offset, value) for primer1
 * (engine.py:331-355); pcr_size is the adjusted expected size (engine.py:245-247).
 * primer1/primer2 bytes are the upper-cased primers of each record ('-' records
 * carry primer2 = reverse complement, engine.py:272-279), concatenated, with
 * CSR offsets p1_off[n_rec+1] / p2_off[n_rec+1].  Bytes >= 0x80 are opaque codes
 * that match only an identical genome byte. */
int mp_table_create(const mp_params* params, int32_t device, uint32_t n_rec,
                    const uint32_t* key, const uint32_t* hash_off,
                    const uint64_t* pcr_size,
                    const uint8_t* primer1, const uint64_t* p1_off,
                    const uint8_t* primer2, const uint64_t* p2_off,
                    void** table_out);
/* Table statistics: distinct keys, largest bucket, device bytes. */
int mp_table_stats(void* table, uint64_t* n_keys, uint64_t* max_bucket, uint64_t* dev_bytes);
/* Split seeds of a W 7..9, I = 0, N <= 1 table (the dense table's search as 11-base exact-seed
 * scans, mp_internal.h kSplitSeed): seed_tables = 0 (not split), 1 (the contiguous seed, N = 0) or 2
 * (contiguous + gapped, N = 1); rest_records = records left to the dense scan. */
int mp_table_split(void* table, uint32_t* seed_tables, uint32_t* rest_records);
/* Which seed structures the table holds (what its scans will take), as MP_LAYOUT_* bits. */
#define MP_LAYOUT_LDS_EXACT 1u /* the LDS prefilter is the exact 4^W bitmap (W <= 10) */
#define MP_LAYOUT_RANK 2u      /* rank words + bucket heads (W <= 13) */
#define MP_LAYOUT_KGRP 4u      /* key groups, one u64 per 16 keys (W 11..13) */
#define MP_LAYOUT_KGRP4 8u     /* wide I = 1 key groups, one 16-B word per 32 keys */
#define MP_LAYOUT_DENSE 16u    /* dense_kernel structures (W <= 9) */
#define MP_LAYOUT_SPLIT 32u    /* split seeds (mp_table_split) */
#define MP_LAYOUT_HASHED 64u   /* hashed presence filter + open-addressed slots (W >= 14) */
#define MP_LAYOUT_DEFER_FULL 128u /* full-head buckets deferred to tail_kernel; the I = 0 key-group
                                     scan forms (and their 16-B key references) need it */
int mp_table_layout(void* table, uint32_t* flags);
/* Layout choices of a table build.  Every field zero = the library's own choice (what
 * mp_table_create makes); the others exist for A/B runs and for tests that drive each layout
 * against the oracle.  No layout choice is read from the process environment. */
typedef struct mp_table_options {
    int32_t lds_k;   /* W 11..13: prefilter bits per key, 1..3; 0 = from the key count */
    int32_t no_h12;  /* 1: IUPAC-after-seed tables keep the 16-B heads, not the 8-B IUPAC heads */
    int32_t kgrp4;   /* wide I = 1 key groups: 0 = when the pass-rate estimate favours them,
                        1 = never, -1 = whenever the table can carry them */
    int32_t no_split;/* 1: W 7..9 tables are not split into exact-seed sub-tables */
} mp_table_options;
int mp_table_create_ex(const mp_params* params, int32_t device, uint32_t n_rec,
                       const uint32_t* key, const uint32_t* hash_off,
                       const uint64_t* pcr_size,
                       const uint8_t* primer1, const uint64_t* p1_off,
                       const uint8_t* primer2, const uint64_t* p2_off,
                       const mp_table_options* options, void** table_out);
void mp_table_destroy(void* table);

/* ---- genome (replaces the per-record sequence strings that search() walks,
 * engine.py:373-411, after FASTALoader filtering, fasta.py:60) ---------------
 * Sequences are resident in HBM as a 2-bit plane + two 1-bit exception planes
 * (0.375 B/base) + a sparse index of non-ACGT runs. */
int mp_genome_create(int32_t device, uint32_t n_seq, const uint64_t* seq_len, void** genome_out);
/* Pack bytes [offset, offset+nbytes) of sequence `seq` from HOST memory.  offset
 * must be a multiple of 64.  Lower-case a-z is upper-cased (engine.py:455). */
int mp_genome_put(void* genome, uint32_t seq, uint64_t offset, const uint8_t* host_bytes,
                  uint64_t nbytes, void* stream);
/* Same, from DEVICE memory on the genome's device. */
int mp_genome_put_device(void* genome, uint32_t seq, uint64_t offset, const uint8_t* dev_bytes,
                         uint64_t nbytes, void* stream);
/* Build the exception-run index; required once after the last put. */
int mp_genome_seal(void* genome, void* stream);
int mp_genome_stats(void* genome, uint64_t* total_bases, uint64_t* n_exc_runs, uint64_t* dev_bytes);
/* Diagnostic (tests): copy the packed planes of a sealed genome to host memory -- g2
 * (total/32 words), gexc, ginv and gwild (total/64 words each; total = padded bases, the sum
 * of each length rounded up to 64) and the sorted exception-run index (n_exc_runs starts and
 * characters).  Any pointer may be NULL to skip that array. */
int mp_genome_download(void* genome, uint64_t* g2, uint64_t* gexc, uint64_t* ginv, uint64_t* gwild,
                       uint64_t* xr_start, uint8_t* xr_char);
/* Re-lay the handle out for a new set of sequences (the next search() call of the
 * engine): device planes are reused when the new layout fits them, else regrown.  The
 * handle is unsealed and empty afterwards; searches created on it stay valid. */
int mp_genome_reset(void* genome, uint32_t n_seq, const uint64_t* seq_len);
void mp_genome_destroy(void* genome);

/* ---- search (replaces _process_thread/_match_sts/_compare_seqs and the
 * sort of engine.py:434; T=1 semantics) ---------------------------------------
 * A search handle owns the hit buffers for one (table, genome) pair. */
int mp_search_create(void* table, void* genome, void** search_out);

/* Kernel-path selection and initial list capacities of a search handle.  Every field
 * zero (the state after mp_search_create) = the library's own choice; the other values
 * exist so that tests can drive each path of the hot loop and its overflow recovery. */
#define MP_TAILS_AUTO 0    /* bucket tails: chosen from the table's key sharing */
#define MP_TAILS_INLINE 1  /* expanded by the scanning wave itself */
#define MP_TAILS_KERNEL 2  /* left as references for tail_kernel */
#define MP_SORT_AUTO 0     /* device bucket sort when the order key fits 64 bits */
#define MP_SORT_RADIX64 1  /* rocPRIM radix sort of the packed 64-bit key */
#define MP_SORT_RADIX128 2 /* two stable rocPRIM passes over the 128-bit key */
#define MP_SORT_SCATTER 3  /* device bucket sort starting from the scatter form (order mode 1) */
typedef struct mp_search_options {
    int32_t tails;              /* MP_TAILS_* */
    int32_t no_defer;           /* 1: the ranked drain tests full-head buckets itself */
    int32_t no_dense;           /* 1: W <= 9 tables run scan_kernel, not dense_kernel */
    int32_t sort;               /* MP_SORT_* */
    int32_t sort_bucket_bits;   /* device bucket sort: log2(buckets); 0 = from the capacity */
    int32_t pair_blocks_per_cu; /* pair_kernel residency; 0 = every resident slot */
    uint64_t hit_cap;           /* initial raw-hit list capacity (entries); 0 = default */
    uint64_t surv_cap;          /* initial fingerprint-survivor list capacity; 0 = default */
    uint64_t tail_cap;          /* initial bucket-tail reference list capacity; 0 = default */
    int32_t no_rank_filter;     /* 1: level-2 probes read the plain rank bitmap, without the
                                   filtered rank groups' primer-base filter */
    int32_t no_split;           /* 1: W 7..9 tables keep the dense scan, not the split seeds
                                   (two exact-seed scans, see mp_internal.h kSplitSeed) */
    int32_t generic_forms;      /* MP_GENERIC_* bits: the run-time-shape kernel forms in place of
                                   the constant-shape ones (A/B; the hit lists are identical) */
    int32_t ref32;              /* 1: 32-B bucket-tail key references where 16-B ones fit */
    int32_t sched_short;        /* super-steps per scheduler claim in short scans; 0 = 4 */
    int32_t crowd_grid;         /* workgroups of the crowded-bucket sort; 0 = one per CU */
    int32_t scan_grid;          /* scan_kernel workgroups; 0 = one per CU.  Fewer leave CUs free
                                   for another pipelined run's post-scan kernels */
} mp_search_options;
#define MP_GENERIC_FIX 1u   /* key-group scans of W = 11 with W, F and N as run-time values */
#define MP_GENERIC_GAP 2u   /* the gapped W = 8 split seed with its shape as run-time values */
#define MP_GENERIC_PAIR 4u  /* pair_kernel with I, N and X as run-time values */
/* Replace the handle's options (reallocating the lists to the given capacities). */
int mp_search_set_options(void* search, const mp_search_options* opt);
/* Per-stage timing (tail, pair and order events; default on).  Off, a run records only the
 * scan kernel's two events: each event between two kernels idles the GPU ~6 us. */
int mp_search_set_stage_timing(void* search, int32_t on);
/* Scan kernel timing (its two HIP events, default on).  Off, mp_search_last_stats reports
 * scan_ms = -1 and the run carries no event before the scan and none after it. */
int mp_search_set_scan_timing(void* search, int32_t on);
/* Scan, verify, pair-check and sort.  *n_hits receives the number of hits of
 * the owned range (range NULL = whole genome).  Waits for the run (= enqueue + complete). */
int mp_search_run(void* search, const mp_range* range, void* stream, uint64_t* n_hits);
/* The asynchronous form: enqueue every kernel of a run on `stream` and return without
 * waiting (the first run of a range uploads its spans).  Other work -- another search
 * handle's run, a collective -- may be enqueued before mp_search_complete, which waits for
 * it, regrows and reruns a list that overflowed, and reports the hit count.  One run per
 * handle may be pending; the handle's hit buffers belong to it until completed. */
int mp_search_enqueue(void* search, const mp_range* range, void* stream);
int mp_search_complete(void* search, uint64_t* n_hits);
/* Copy the sorted hits of the last run to host memory (cap entries). */
int mp_search_fetch(void* search, mp_hit* out, uint64_t cap, void* stream);
/* Copy the sorted hits of the last run into DEVICE memory on the search's GPU
 * (e.g. a communication buffer for the multi-GPU gather). */
int mp_search_fetch_device(void* search, mp_hit* dev_out, uint64_t cap, void* stream);
/* Device pointer to the sorted hits of the last run (n_hits entries of mp_hit). */
int mp_search_device_hits(void* search, const mp_hit** dev_hits);
/* Duration of the last run's scan kernel alone (HIP events on the run's stream), the
 * number of candidate seeds it verified and the windows it scanned. */
int mp_search_last_stats(void* search, float* scan_ms, uint64_t* n_windows, uint64_t* n_candidates);
/* List regrowths (a run whose survivor, tail or hit list overflowed and was rerun)
 * over the handle's life. */
int mp_search_regrowths(void* search, uint64_t* n_regrowths);
/* Device bytes the handle holds: hit, survivor and tail lists, sort buffers and the
 * order-mode-0 bucket slots (which grow with the hit capacity's bucket plan). */
int mp_search_dev_bytes(void* search, uint64_t* dev_bytes);
/* Seeds whose primer-1 fingerprint could not reject them (pair-checked). */
int mp_search_survivors(void* search, uint64_t* n_survivors);
/* Last run's stage times (HIP events on the run's stream): seed scan kernel alone,
 * bucket-tail kernel, survivor pair-check kernel, ordering (sort + decode). */
int mp_search_timing(void* search, float* scan_ms, float* tail_ms, float* pair_ms, float* order_ms);
void mp_search_destroy(void* search);

/* ---- multi-GPU (replaces the -T ProcessPool fan-out over chunks of a record,
 * engine.py:386-422) --------------------------------------------------
 * One process, several devices: the genome's (sequence, k) space is split into owned
 * ranges of equal base count, one per device (contiguous, in device order); each device
 * packs only the bases its range reads and searches it in a host thread of its own; the
 * sorted per-device lists are gathered into devices[0] by the copy engines over xGMI
 * (mp_multi_set_gather).  Their concatenation is exactly the single-device hit list.
 * tables[i] must have been created on devices[i] from the same records.  A device may be
 * listed twice (tests on one GPU): the gather is the same peer copy. */
int mp_multi_create(uint32_t n_dev, const int32_t* devices, void* const* tables, void** multi_out);
/* (Re)lay out the sequence set on every device and split it into owned ranges. */
int mp_multi_genome(void* multi, uint32_t n_seq, const uint64_t* seq_len);
/* Whole sequence `seq` from host memory (each device packs its share + halo). */
int mp_multi_put(void* multi, uint32_t seq, const uint8_t* host_bytes, uint64_t nbytes);
int mp_multi_seal(void* multi);
/* Search every device's owned range and gather: *n_hits = all hits, in output order. */
int mp_multi_run(void* multi, uint64_t* n_hits);
/* The gather's data plane.  MP_GATHER_COPY (default): the copy engines move each device's
 * sorted list into devices[0] (hipMemcpyPeerAsync on devices[0]'s stream, peer access enabled
 * once; no kernel on the CUs), for distinct and repeated devices alike.  MP_GATHER_RCCL: one
 * grouped ncclSend/ncclRecv gatherv (ncclCommInitAll at the first such run; distinct devices
 * only). */
#define MP_GATHER_COPY 0
#define MP_GATHER_RCCL 1
int mp_multi_set_gather(void* multi, int32_t mode);
int mp_multi_fetch(void* multi, mp_hit* out, uint64_t cap);
/* Device i's search handle (borrowed: stats, timings), its owned range and the last
 * gather's duration on devices[0]'s stream. */
int mp_multi_device_search(void* multi, uint32_t i, void** search, mp_range* owned, float* gather_ms);
/* The last mp_multi_run's device span on devices[0] (its start, before the first search is
 * enqueued, to the gather's end) and the gather alone; wall time minus the span is the host
 * overhead of the call. */
int mp_multi_timing(void* multi, float* span_ms, float* gather_ms);
void mp_multi_destroy(void* multi);

/* One process per GPU (torchrun-style launch): every rank creates a communicator from an
 * RCCL unique id that rank 0 made (mp_comm_unique_id, 128 bytes) and the caller shared
 * out of band; mp_comm_gather_hits then gathers each rank's last mp_search_run result to
 * rank 0 (dev_out on rank 0's device, cap entries), in rank order, adding seq_shift to each
 * rank's sequence indices.  Collective; *n_total = all ranks' hits, on every rank. */
int mp_comm_unique_id(uint8_t* id128);
int mp_comm_create(const uint8_t* id128, int32_t nranks, int32_t rank, int32_t device, void** comm_out);
int mp_comm_gather_hits(void* comm, void* search, uint32_t seq_shift, mp_hit* dev_out, uint64_t cap,
                        uint64_t* n_total, void* stream);
void mp_comm_destroy(void* comm);

/* One node, one process per GPU, no kernel on the CUs: rank 0 exports its gather buffer and
 * count words once (mp_ipc_handle, MP_IPC_HANDLE_BYTES each, shared out of band), every rank
 * maps them (mp_ipc_open on its own device; rank 0 may use its pointers directly) and after
 * each completed run mp_search_put_hits copies the run's hits into its region of that buffer
 * and the count into its count word, on `stream`, by the copy engines
 * (hipMemcpyDeviceToDeviceNoCU / host-to-device): a persistent scan holds every CU's LDS, so a
 * collective's kernels (RCCL's need 37 KiB of LDS) would wait for the scan to end.  Regions
 * are fixed: rank r owns [r * cap, (r + 1) * cap) entries; a sequence-index shift (contig
 * shards) is the reader's.  *n_hits (may be NULL) = the run's hit count, always: on MP_E_CAP
 * (more hits than cap, nothing copied) it is the region size a regrow needs.  Not collective;
 * completion is the stream's.  The handle's next mp_search_enqueue, on any stream, waits on the
 * device for the put to have read the hit list; a handle's puts must stay on one stream. */
#define MP_IPC_HANDLE_BYTES 64
/* The handle names dev_ptr's whole allocation; *offset = dev_ptr - its base.  mp_ipc_open
 * returns the base as mapped here: add the offset. */
int mp_ipc_handle(void* dev_ptr, uint8_t* handle64, uint64_t* offset);
int mp_ipc_open(const uint8_t* handle64, int32_t device, void** base_out);
int mp_ipc_close(void* dev_ptr);
int mp_search_put_hits(void* search, mp_hit* dst, uint64_t cap, uint64_t* count_dst, uint64_t* n_hits,
                       void* stream);

/* ---- FASTA input (replaces FASTALoader.load_file, src/merpcr/io/fasta.py:18-71) --
 * Reads `path` as the reference's text-mode loop does: strict UTF-8, universal
 * newlines, Python str.strip() whitespace, '>' headers (defline = stripped line),
 * sequence lines filtered to the characters whose upper case is in
 * "ACGTBDHKMNRSVWXY" (32 ASCII letters + U+017F as its two UTF-8 bytes), lines
 * before the first header dropped.  The caller handles the reference's empty-file
 * case (fasta.py:31-33) before calling.  Records stay owned by the handle. */
int mp_fasta_load(const char* path, void** fasta_out);
/* Same rules over the memory-mapped file on `threads` host threads (0 = every CPU the
 * process may use; mp_fasta_load's choice): UTF-8 validation, header lines and the
 * filter each split over the threads.  An unmappable file falls back to the streaming
 * reader below. */
int mp_fasta_load_parallel(const char* path, int32_t threads, void** fasta_out);
/* The streaming reader, one thread, reading the file in chunks of `chunk_bytes` (0 = 64
 * MiB): tests use small chunks to put read seams inside lines, UTF-8 sequences and CR/LF
 * pairs. */
int mp_fasta_load_chunked(const char* path, uint64_t chunk_bytes, void** fasta_out);
/* Number of records and total filtered sequence bytes. */
int mp_fasta_info(void* fasta, uint64_t* n_records, uint64_t* total_bytes);
/* Borrowed pointers to record i's defline (UTF-8, with '>') and filtered sequence. */
int mp_fasta_record(void* fasta, uint64_t i, const uint8_t** defline, uint64_t* defline_len,
                    const uint8_t** seq, uint64_t* seq_len);
/* 1 when record i's filtered sequence is ASCII (no U+017F), else 0. */
int mp_fasta_record_ascii(void* fasta, uint64_t i, int32_t* ascii);
void mp_fasta_destroy(void* fasta);
/* Device ingestion of an ASCII FASTA file (the same records as mp_fasta_load): the raw
 * bytes are uploaded to `device` and the header search, the keep-set filter
 * (fasta.py:42-66) and the compaction run there; the filtered sequences stay in device
 * memory, record after record (mp_fasta_device_info's dev_bases), ready for
 * mp_genome_put_device.  *ascii = 0 and no handle when the file holds a byte >= 0x80 (or
 * more than 2^20 header lines): read it with mp_fasta_load. */
int mp_fasta_load_device(const char* path, int32_t device, void* stream, void** fasta_out, int32_t* ascii);
int mp_fasta_device_info(void* fasta, uint64_t* n_records, uint64_t* total_bases, const uint8_t** dev_bases);
/* Record i: its stripped defline and its bases' offset and length in dev_bases. */
int mp_fasta_device_record(void* fasta, uint64_t i, const uint8_t** defline, uint64_t* defline_len,
                           uint64_t* offset, uint64_t* length);
/* Bases [offset, offset + n) of dev_bases into host memory. */
int mp_fasta_device_read(void* fasta, uint64_t offset, uint64_t n, uint8_t* host_dst);
void mp_fasta_device_destroy(void* fasta);

/* ---- STS file (replaces MerPCR.load_sts_file and helpers, engine.py:193-359) --
 * Parses `path` into the oriented records of the reference's sts_records, in order,
 * with the same skip/adjust rules.  The caller handles the empty-file case
 * (engine.py:196-200).  Status after a successful parse: */
#define MP_STS_OK 0        /* whole file parsed */
#define MP_STS_BAD_LINE 1  /* stopped at a line with < 4 fields (load returns False);
                              the records before it are kept, as in the reference */
#define MP_STS_PYTHON 2    /* a primer/size field needs Python's Unicode upper()/int()
                              rules (non-ASCII) or a size >= 2^62: parse on the host side */
int mp_sts_parse(const char* path, int32_t wordsize, int64_t default_pcr_size, void** sts_out);
/* counts[10]: n_records, bad_line, n_short, n_ambig, n_badsize, max_pcr_size,
 * primer1 bytes, primer2 bytes, text bytes, n_text (= 2 x kept lines). */
int mp_sts_info(void* sts, int32_t* status, uint64_t* counts);
/* ptrs[12] (borrowed, valid until destroy): key u32[n], hash_off u32[n], pcr_size u64[n],
 * line_no u64[n], direct u8[n] ('+'/'-'), text_idx u32[n] (line index: id = text item
 * 2i, alias = 2i+1), primer1 u8[], p1_off u64[n+1], primer2 u8[], p2_off u64[n+1],
 * text u8[] (UTF-8), text_off u64[n_text+1]. */
int mp_sts_arrays(void* sts, const void** ptrs);
/* The formatter's record column (mp_format_hits rec_text / rec_off) of the parsed
 * records: UTF-8 "{id}\t{alias}\t({direct})" per record, concatenated (*n_bytes), with
 * n+1 offsets.  Borrowed, valid until destroy. */
int mp_sts_record_texts(void* sts, const uint8_t** text, const uint64_t** off, uint64_t* n_bytes);
void mp_sts_destroy(void* sts);

/* ---- output (replaces the per-hit print of MerPCR.search, engine.py:436-444) --
 * Writes one line per hit, in the order given:
 *     "{label}\t{pos1+1}..{pos2+1}\t{rec_text}\n"
 * labels: UTF-8 FASTARecord.label of each sequence, CSR offsets label_off[n_seq+1];
 * rec_text: UTF-8 "{id}\t{alias}\t({direct})" of each record in sts_records order,
 * CSR offsets rec_off[n_rec+1].  *n_bytes receives the output size; out == NULL is a
 * size query, cap < size fails with MP_E_CAP. */
int mp_format_hits(const mp_hit* hits, uint64_t n_hits,
                   const uint8_t* labels, const uint64_t* label_off, uint32_t n_seq,
                   const uint8_t* rec_text, const uint64_t* rec_off, uint32_t n_rec,
                   uint8_t* out, uint64_t cap, uint64_t* n_bytes);

#ifdef __cplusplus
}
#endif
#endif /* MERPCR_HIP_H */
