// Internal declarations shared by the product sources: the WAL scan object
// (GPU scan + host reader) and the lv_last_error plumbing.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace lvgpu_internal {
// One block-aligned chunk of a pipelined scan (offsets are log offsets).
struct ScanChunk {
    std::vector<uint64_t> off;
    std::vector<uint32_t> crc, info;
};
// A scan still running (lv_wal_scan_host_pipelined): a worker thread scans
// the log's chunks in order; readers wait for the chunk they need.
struct ScanPipe {
    std::vector<uint64_t> lo;  // chunk k is log[lo[k], lo[k + 1]) (block-aligned; lo.back() = the log size)
    std::vector<ScanChunk> chunks;
    std::mutex m;
    std::condition_variable cv;
    size_t ready = 0;  // chunks [0, ready) are complete (all of them once rc != 0)
    std::atomic<size_t> ready_seen{0};  // `ready`, read without the lock (set after it)
    int rc = 0;
    std::string err;
    std::thread worker;
    bool flat = false;  // the scan's flat arrays were filled
    // 0 once chunk k is complete, or the worker's error
    int wait(size_t k) {
        if (ready_seen.load(std::memory_order_acquire) > k) return 0;  // the Reader's per-record path
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return ready > k || rc != 0; });
        return ready > k ? 0 : rc;
    }
    ~ScanPipe() {
        if (worker.joinable()) worker.join();
    }
};
}  // namespace lvgpu_internal

struct lv_wal_scan {
    std::vector<uint64_t> off;   // physical-record header offsets, ascending
    std::vector<uint32_t> crc;   // value([type || payload]) (0 unless status OK)
    std::vector<uint32_t> info;  // type | status << 8 | payload_length << 16
    // lv_wal_scan_host_pipelined: the chunks still arriving (the flat arrays
    // above are filled from them when first asked for), or null
    std::unique_ptr<lvgpu_internal::ScanPipe> pipe;
};

namespace lvgpu_internal {
int set_error(int code, const char *msg);  // lv_last_error plumbing (context.hip)
void clear_error();
int launch_status();                       // hipGetLastError -> LV status + message

// Selects a device for the calling thread and restores the thread's previous
// current device when it goes out of scope: the host entry points take a
// `device` argument, and a drop-in C ABI must not leave the caller's thread
// pointed at another GPU (context.hip).
struct DeviceGuard {
    int prev = -1;
    DeviceGuard() = default;
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
    int set(int device);  // LV status; the first call saves the current device
    ~DeviceGuard();
};

// Scan of log[0, bytes) on `device` into `out` (offsets += base): the body of
// lv_wal_scan_host, one chunk of a pipelined scan (wal_scan.hip).
int scan_host_range(const uint8_t *log, size_t bytes, uint64_t base, int device, ScanChunk *out);
// Waits for a pipelined scan and fills its flat arrays (no-op otherwise).
int scan_flatten(lv_wal_scan *scan);

// Host-memory path of one device (context.hip): holds the device's
// host-path lock while alive.  host_upload copies `bytes` of host memory into
// the device's cached arena (pinned input: one DMA; pageable: a pipelined
// pinned staging copy) followed by `pad` zero bytes, on the device's stream.
struct HostPath {
    DeviceGuard dg;  // restored after the lock is released
    std::unique_lock<std::mutex> lk;
    void *stream = nullptr;     // hipStream_t
    uint8_t *d_arena = nullptr;
};
int host_upload(int device, const uint8_t *h, size_t bytes, size_t pad, HostPath *hp);
// SSTable trailer seal (d_types may be NULL) or verify (d_status, optional
// d_crc) of n blocks in one launch on the current device (sst.hip).
int launch_sst_blocks(bool seal, const uint8_t *d_file, uint64_t file_bytes, const uint64_t *d_handles,
                      const uint8_t *d_types, size_t n, uint32_t *d_status, uint32_t *d_crc, void *stream);
// Cached device scratch buffer `slot` (0..1) of the HostPath's device, >= bytes.
int host_scratch(HostPath *hp, int slot, size_t bytes, uint8_t **d);
// Page-locked host memory (hipHostMalloc): a buffer host_upload DMAs in one
// copy, with no staging pass.
int pinned_alloc(size_t bytes, uint8_t **p);
void pinned_free(uint8_t *p);
// lv_device_counters bookkeeping for host copies made outside
// context.hip (current device).
void count_h2d(uint64_t bytes);
void count_d2h(uint64_t bytes);
// ... and an allocation the host path made for `device` (any thread).
void count_alloc(int device);
}
