/*
 * Timing helper for bench.py --wal (VERDICT r03 "next" 8): the reference
 * Reader loop as a Rust caller of the C ABI would run it -- lv_wal_reader_new
 * over a log and its GPU scan, then lv_wal_reader_read_record until the end
 * of input (log_reader.rs:120-265), in one C loop with no per-record FFI
 * hop.  Not part of the product library; built beside it by
 * leveldb-rs_amd/Makefile into lib/libhostreplay.so and loaded by bench.py.
 */
#include <stddef.h>
#include <stdint.h>
#include <time.h>

#include "../include/lvgpu/wal.h"

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* The recovery pass end to end as a native caller runs it (VERDICT r04
 * missing 3): lv_wal_scan_host_pipelined, the Reader loop over it (replaying
 * chunk k while chunk k + 1 is scanned), lv_wal_scan_free; best of `reps`
 * passes, records / payload bytes of one pass (-1.0 on an error). */
double lv_replay_recover(const uint8_t *log, size_t bytes, int device, int reps, uint64_t *records,
                         uint64_t *payload) {
    double best = -1.0;
    for (int r = 0; r < reps; ++r) {
        const double t0 = now_s();
        lv_wal_scan *scan = lv_wal_scan_host_pipelined(log, bytes, device);
        if (!scan) return -1.0;
        lv_wal_reader *rd = lv_wal_reader_new(log, bytes, scan, NULL, NULL, 1, 0);
        if (!rd) return -1.0;
        uint64_t n = 0, b = 0;
        const uint8_t *d = NULL;
        size_t len = 0;
        int rc;
        while ((rc = lv_wal_reader_read_record(rd, &d, &len)) == 1) {
            ++n;
            b += len;
        }
        lv_wal_reader_free(rd);
        lv_wal_scan_free(scan);
        const double el = now_s() - t0;
        if (rc < 0) return -1.0;
        if (best < 0 || el < best) best = el;
        *records = n;
        *payload = b;
    }
    return best;
}

/* The pipelined scan alone: lv_wal_scan_host_pipelined, lv_wal_scan_wait,
 * lv_wal_scan_free; best of `reps` (-1.0 on an error). */
double lv_replay_scan_pipelined(const uint8_t *log, size_t bytes, int device, int reps) {
    double best = -1.0;
    for (int r = 0; r < reps; ++r) {
        const double t0 = now_s();
        lv_wal_scan *scan = lv_wal_scan_host_pipelined(log, bytes, device);
        if (!scan) return -1.0;
        const int rc = lv_wal_scan_wait(scan);
        lv_wal_scan_free(scan);
        const double el = now_s() - t0;
        if (rc) return -1.0;
        if (best < 0 || el < best) best = el;
    }
    return best;
}

/* Replays the whole log `reps` times; returns the best pass in seconds and
 * the records / payload bytes of one pass (-1.0 on a reader error). */
double lv_replay_reader(const uint8_t *log, size_t bytes, const lv_wal_scan *scan, int reps, uint64_t *records,
                        uint64_t *payload) {
    double best = -1.0;
    for (int r = 0; r < reps; ++r) {
        const double t0 = now_s();
        lv_wal_reader *rd = lv_wal_reader_new(log, bytes, scan, NULL, NULL, 1, 0);
        if (!rd) return -1.0;
        uint64_t n = 0, b = 0;
        const uint8_t *d = NULL;
        size_t len = 0;
        int rc;
        while ((rc = lv_wal_reader_read_record(rd, &d, &len)) == 1) {
            ++n;
            b += len;
        }
        lv_wal_reader_free(rd);
        const double el = now_s() - t0;
        if (rc < 0) return -1.0;
        if (best < 0 || el < best) best = el;
        *records = n;
        *payload = b;
    }
    return best;
}
