// Kernel tuning parameters (LVK_*) of the product library.
//
// The defaults below ARE the product: each is a parameter a kept sweep varies
// (tools/ab_lib.sh, tools/r06/*.sh) with the measured alternatives documented
// where it is used, and the GPU suite tests the kernels only at these values.
// (Round 6 removed the switches whose alternatives were measured and settled,
// with their code paths, and the timing-only switches that computed wrong
// CRCs.)  Setting any of them is therefore an error
// unless the build declares itself an experiment variant: tools/build_variant.sh
// defines LVK_EXPERIMENT_BUILD and writes the library to lib/variants/, which
// never ships to the GPU box and which the Python binding loads only with
// LVGPU_EXPERIMENT=1.  tests/test_abi.py checks that every switch is listed
// in the guard.
#pragma once

#if !defined(LVK_EXPERIMENT_BUILD) && ( \
    defined(LVK_STAGGER) || \
    defined(LVK_AL_ROWS) || \
    defined(LVK_MAX_PIECES) || \
    defined(LVK_WAL_TOUCH_HOPS) || \
    defined(LVK_SMALL_WAVES) || \
    defined(LVK_SEAL_FLUSH) || \
    defined(LVK_SST_ROWS) || \
    defined(LVK_SEAL_ROWS) || \
    defined(LVK_SST_RUN) || \
    defined(LVK_SORT_MIN_WGS) || \
    defined(LVK_SMALL_ROUNDS) || \
    defined(LVK_HASH_WGS_PER_CU) || \
    defined(LVK_PIPE_CHUNK_MB) || \
    defined(LVK_PIPE_FIRST_MB) || \
    defined(LVK_MEMCPY_THREADS) || \
    defined(LVK_PIPE_COPY_THREADS) || \
    defined(LVK_WAL_UNSORT))
#error "LVK_* kernel switches select untested code paths; only experiment variants (LVK_EXPERIMENT_BUILD, tools/build_variant.sh) may set them"
#endif

#ifndef LVK_STAGGER  // s_sleep(32) units between the start of successive waves (blocks kernel, >= 8 KiB)
#define LVK_STAGGER 1u
#endif
#ifndef LVK_AL_ROWS
#define LVK_AL_ROWS 4
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
#ifndef LVK_SMALL_ROUNDS  // small-class rounds per wave (round 4, after the unsort: 52 over 26: C2 +0.4 %, C4 +0.6 %)
#define LVK_SMALL_ROUNDS 52
#endif
#ifndef LVK_PIPE_CHUNK_MB  // host: chunk of the pipelined WAL scan (MiB, block multiple)
#define LVK_PIPE_CHUNK_MB 32
#endif
#ifndef LVK_PIPE_FIRST_MB  // host: the pipelined WAL scan's first chunk (MiB; the chunks double up to LVK_PIPE_CHUNK_MB)
#define LVK_PIPE_FIRST_MB 2
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
