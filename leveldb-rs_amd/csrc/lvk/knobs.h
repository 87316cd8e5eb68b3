// Kernel tuning switches (LVK_*) of the product library.
//
// The defaults below ARE the product: each switch records a measured
// alternative (documented where it is used), and the GPU suite tests the
// kernels only at these values.  Setting any of them is therefore an error
// unless the build declares itself an experiment variant: tools/build_variant.sh
// defines LVK_EXPERIMENT_BUILD and writes the library to lib/variants/, which
// never ships to the GPU box and which the Python binding loads only with
// LVGPU_EXPERIMENT=1.  tests/test_abi.py checks that every switch is listed
// in the guard.
#pragma once

#if !defined(LVK_EXPERIMENT_BUILD) && ( \
    defined(LVK_EXP_NOSHIFT) || \
    defined(LVK_EXP_NOFOLD) || \
    defined(LVK_STAGGER) || \
    defined(LVK_EXP_NOSTAGE) || \
    defined(LVK_EXP_NOTAIL) || \
    defined(LVK_EXP_NOFIX) || \
    defined(LVK_EXP_NOMERGE) || \
    defined(LVK_EXP_NOSEALWRITE) || \
    defined(LVK_EXP_NOOUT) || \
    defined(LVK_EXP_SORTEDOUT) || \
    defined(LVK_AL_ROWS) || \
    defined(LVK_ALIGNED_ROWS) || \
    defined(LVK_IDENT) || \
    defined(LVK_MAX_PIECES) || \
    defined(LVK_WAL_TOUCH_HOPS) || \
    defined(LVK_SMALL_WAVES) || \
    defined(LVK_SMALL_ALL) || \
    defined(LVK_CLASS_STAGGER) || \
    defined(LVK_SEAL_FLUSH) || \
    defined(LVK_SST_ROWS) || \
    defined(LVK_SEAL_ROWS) || \
    defined(LVK_SST_RUN) || \
    defined(LVK_SORT_MIN_WGS) || \
    defined(LVK_CLASS3_FIRST) || \
    defined(LVK_SMALL_ADAPT) || \
    defined(LVK_SMALL_ROUNDS) || \
    defined(LVK_FUSED_ONE_ROUND) || \
    defined(LVK_FUSED_LOCAL_JOIN) || \
    defined(LVK_EXP_SEAL_COMPACT) || \
    defined(LVK_HASH_SPAN_READLANE) || \
    defined(LVK_HASH_WGS_PER_CU) || \
    defined(LVK_HASH_PREFETCH_EXACT) || \
    defined(LVK_EXP_HASH_MUL24) || \
    defined(LVK_HASH_TAIL_READ) || \
    defined(LVK_HASH_LDS_ALL) || \
    defined(LVK_PIPE_CHUNK_MB) || \
    defined(LVK_MEMCPY_THREADS) || \
    defined(LVK_PIPE_COPY_THREADS) || \
    defined(LVK_WALK_EXACT) || \
    defined(LVK_WAL_UNSORT) || \
    defined(LVK_TABLE_EXACT) || \
    defined(LVK_FUSED_EXACT))
#error "LVK_* kernel switches select untested code paths; only experiment variants (LVK_EXPERIMENT_BUILD, tools/build_variant.sh) may set them"
#endif

#ifndef LVK_EXP_NOSHIFT
#define LVK_EXP_NOSHIFT 0
#endif
#ifndef LVK_EXP_NOFOLD
#define LVK_EXP_NOFOLD 0
#endif
#ifndef LVK_STAGGER  // s_sleep(32) units between the start of successive waves (blocks kernel, >= 8 KiB)
#define LVK_STAGGER 1u
#endif
#ifndef LVK_EXP_NOSTAGE
#define LVK_EXP_NOSTAGE 0
#endif
#ifndef LVK_EXP_NOTAIL
#define LVK_EXP_NOTAIL 0
#endif
#ifndef LVK_EXP_NOFIX
#define LVK_EXP_NOFIX 0
#endif
#ifndef LVK_EXP_NOMERGE
#define LVK_EXP_NOMERGE 0
#endif
#ifndef LVK_EXP_NOSEALWRITE  // the seal computes its trailers but stores none
#define LVK_EXP_NOSEALWRITE 0
#endif
#ifndef LVK_EXP_NOOUT  // timing only: the class kernel computes its CRCs but stores none
#define LVK_EXP_NOOUT 0
#endif
#ifndef LVK_EXP_SORTEDOUT  // timing only: the class kernel stores each CRC at its sorted position (wrong order)
#define LVK_EXP_SORTEDOUT 0
#endif
#ifndef LVK_AL_ROWS
#define LVK_AL_ROWS 4
#endif
#ifndef LVK_ALIGNED_ROWS
#define LVK_ALIGNED_ROWS 1
#endif
#ifndef LVK_IDENT
#define LVK_IDENT 1
#endif
#ifndef LVK_MAX_PIECES  // pieces per split buffer (a lone 16 MiB buffer: 4,096 of 4 KiB, as the strided API cuts it)
#define LVK_MAX_PIECES 4096
#endif
#ifndef LVK_WAL_TOUCH_HOPS
#define LVK_WAL_TOUCH_HOPS 16
#endif
#ifndef LVK_SMALL_WAVES
#define LVK_SMALL_WAVES 4
#endif
#ifndef LVK_SMALL_ALL
#define LVK_SMALL_ALL 1
#endif
#ifndef LVK_CLASS_STAGGER
#define LVK_CLASS_STAGGER 1
#endif
#ifndef LVK_SEAL_FLUSH  // rounds per seal flush (<= 16: 64 two-word slots)
#define LVK_SEAL_FLUSH 16
#endif
#ifndef LVK_SST_ROWS  // table walk rows per batch (round 4, verify with exact waits: 4 rows 0.69 vs 3 rows 0.71, profiles/r04/sst_rows/)
#define LVK_SST_ROWS 3
#endif
#ifndef LVK_SEAL_ROWS  // the seal's rows per batch: LVK_SST_ROWS, or 4 on the G = 16 image
#define LVK_SEAL_ROWS LVK_SST_ROWS
#endif
#ifndef LVK_SST_RUN  // table walk: consecutive blocks per group (file-order runs; 1 = one block per round)
#define LVK_SST_RUN 4
#endif
#ifndef LVK_SORT_MIN_WGS
#define LVK_SORT_MIN_WGS 1024
#endif
#ifndef LVK_CLASS3_FIRST  // class kernel: walk class 3 (> 32 KiB) before class 2 (SortedList::r3)
#define LVK_CLASS3_FIRST 1
#endif
#ifndef LVK_SMALL_ADAPT  // class kernel: small-class waves per workgroup from the class counts (<= LVK_SMALL_WAVES)
#define LVK_SMALL_ADAPT 1
#endif
#ifndef LVK_SMALL_ROUNDS  // small-class rounds per wave (round 4, after the unsort: 52 over 26: C2 +0.4 %, C4 +0.6 %)
#define LVK_SMALL_ROUNDS 52
#endif
#ifndef LVK_FUSED_ONE_ROUND  // fused small-batch walk: a wave's only round requests all its batches at once
#define LVK_FUSED_ONE_ROUND 1
#endif
#ifndef LVK_FUSED_LOCAL_JOIN  // fused small-batch kernel: one-pass batches join workgroup-local split buffers in place
#define LVK_FUSED_LOCAL_JOIN 1
#endif
#ifndef LVK_HASH_SPAN_READLANE  // hash: a wave's span from its first and last lanes (0: two wave reductions)
#define LVK_HASH_SPAN_READLANE 1
#endif
#ifndef LVK_HASH_LDS_ALL  // hash: the staged fast path reads all 17 window dwords from LDS, unmasked
#define LVK_HASH_LDS_ALL 1
#endif
#ifndef LVK_HASH_TAIL_READ  // hash: the tail word re-read after the chain, not captured in it
#define LVK_HASH_TAIL_READ 1
#endif
#ifndef LVK_EXP_HASH_MUL24  // timing only: the hash chain's multiply as v_mul_u32_u24 (wrong hashes)
#define LVK_EXP_HASH_MUL24 0
#endif
#ifndef LVK_HASH_PREFETCH_EXACT  // hash: the next set's metadata loaded by every lane (clamped), no exec mask
#define LVK_HASH_PREFETCH_EXACT 1
#endif
#ifndef LVK_PIPE_CHUNK_MB  // host: chunk of the pipelined WAL scan (MiB, block multiple)
#define LVK_PIPE_CHUNK_MB 32
#endif
#ifndef LVK_MEMCPY_THREADS  // host: threads of the pageable -> pinned staging copy
#define LVK_MEMCPY_THREADS 8
#endif
#ifndef LVK_PIPE_COPY_THREADS  // host: the same in the pipelined WAL scan's worker (a Reader runs beside it)
#define LVK_PIPE_COPY_THREADS 4
#endif
#ifndef LVK_HASH_WGS_PER_CU  // hash: persistent workgroups (4 waves) per CU
#define LVK_HASH_WGS_PER_CU 8
#endif
#ifndef LVK_WAL_UNSORT  // WAL scan: CRCs stored by sorted position, then written in log order (wal_unsort)
#define LVK_WAL_UNSORT 1
#endif
// sorted_stream wait-count mode per source (walk.h): 0 = exec-masked loads,
// 1 = the same unconditional loads every step, 2 = unconditional loads
// within each path (no re-reads)
#ifndef LVK_WALK_EXACT  // the class kernel's sorted lists (offsets API, WAL scan)
#define LVK_WALK_EXACT 0
#endif
#ifndef LVK_TABLE_EXACT  // the SST table walk's verify (the seal keeps mode 0)
#define LVK_TABLE_EXACT 2
#endif
#ifndef LVK_FUSED_EXACT  // the fused small-batch kernel
#define LVK_FUSED_EXACT 0
#endif
#ifndef LVK_EXP_SEAL_COMPACT  // experiment (no trailers): the seal stores its masked crcs to a per-block array
#define LVK_EXP_SEAL_COMPACT 0
#endif
