// Internal declarations shared by the product sources: the WAL scan object
// (GPU scan + host reader) and the lv_last_error plumbing.
#pragma once
#include <cstdint>
#include <vector>

struct lv_wal_scan {
    std::vector<uint64_t> off;   // physical-record header offsets, ascending
    std::vector<uint32_t> crc;   // value([type || payload]) (0 unless status OK)
    std::vector<uint32_t> info;  // type | status << 8 | payload_length << 16
};

namespace lvgpu_internal {
int set_error(int code, const char *msg);  // lv_last_error plumbing (crc32c_batch.hip)
void clear_error();
int launch_status();                       // hipGetLastError -> LV status + message
}
