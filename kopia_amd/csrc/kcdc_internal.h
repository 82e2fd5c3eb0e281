// Internal declarations shared by the kcdc host code and the HIP kernels.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

namespace kcdc {

constexpr int kWindow = 64;  // splitterSlidingWindowSize, repo/splitter/splitter.go:9

struct Tables {
    uint32_t buz[256];      // rollinghash buzhash32 byte table (GenerateHashes(1))
    uint64_t rk_pol = 0;    // rollinghash rabinkarp64 polynomial (RandomPolynomial(1))
    int rk_shift = 0;       // deg(P) - 8
    uint64_t rk_out[256];   // b * x^(8*63) mod P
    uint64_t rk_mod[256];   // (b * x^deg mod P) | (b << deg)
    uint64_t cooked[607];   // Go math/rand rngCooked (rng.go)
};
// rand.New(rand.NewSource(seed)).Read(p[:n]) (Go math/rand, 7 bytes per Int63).
void gorand_read(int64_t seed, uint8_t* p, uint64_t n);
const Tables& tables();

enum Kind : int32_t { kFixed = 0, kBuzhash = 1, kRabinKarp = 2 };

struct Algo {
    const char* name;
    Kind kind;
    bool pooled;
    uint64_t avg;
    uint64_t min_size() const { return kind == kFixed ? avg : avg / 2; }
    uint64_t max_size() const { return kind == kFixed ? avg : avg * 2; }
    uint64_t mask() const { return kind == kFixed ? 0 : avg - 1; }
};
// Registry lookup (repo/splitter/splitter.go:50-86); nullptr if unknown.
const Algo* find_algo(const char* name);
int algo_count();
const Algo* custom_algo(int32_t kind, uint64_t avg);  // interned, nullptr if invalid
int algo_index(const Algo* a);                         // registry index, -1 for custom
const Algo& algo_at(int i);  // sorted by name

// Test knob: lanes per chunk of the content-hash kernels (0 auto, 1, 4).
int& test_hash_lanes();
uint64_t& test_id_ring_bytes();  // kcdc_test_set(KCDC_TEST_ID_RING): the writers' ID ring size (0: default)

// Wrong-output experiment switches compiled into this build (comma-terminated names; "" in
// the product): kcdc_kernels.hip, kcdc_crypt.hip.
const char* ablations_kernels();
const char* ablations_crypt();

// Thread-local error reporting.
int set_error(int code, const std::string& msg);

// ---- kernel launchers (kcdc_kernels.hip) ----
struct DeviceTables;  // per-device copies of the hash tables
const DeviceTables* device_tables(int device, int* err);

struct SplitArgs {
    const uint8_t* const* ptrs;
    const uint64_t* lens;
    uint32_t nstreams;
    uint64_t* cuts;
    uint64_t cuts_cap;
    const uint64_t* cut_base;
    uint64_t* counts;
    const uint64_t* cut_end = nullptr;  // optional per-stream end of the cut range (device)
    const uint64_t* starts = nullptr;   // optional per-stream first chunk start (device; bytes before = history)
    const uint64_t* resume = nullptr;   // optional (with starts): positions below resume[i] are known to hold no
                                        // candidate of stream i's first chunk (a previous round tested them)
};
// Launch the batch splitter for `algo` on `stream` (hipStream_t as void*).
int launch_split_batch(const Algo& algo, const SplitArgs& a, int device, void* stream);
// Single-region first-candidate scan used by the streaming handle:
// bytes [0, len) of `d_buf` are the stream, positions < 0 are zero; returns via
// d_out[0] the first candidate position in [lo, hi] or -1.
// d_scratch (optional, device memory of at least len bytes): copy the bytes there first with
// a whole workgroup, then scan them with 4 waves (for d_buf in mapped host memory).
int launch_scan_first(const Algo& algo, const uint8_t* d_buf, uint64_t len, int64_t lo, int64_t hi, int64_t* d_out,
                      int device, void* stream, uint8_t* d_scratch = nullptr);
// The same scan through the device's resident scan server (no launch): 0 and *out = the
// first candidate in [lo, hi] (or -1); 1 = the server is unavailable or busy (launch
// instead); < 0 = error.  d_stage: fine-grained mapped host memory, 256-byte aligned.
int server_scan_first(const Algo& algo, const uint8_t* d_stage, uint64_t len, int64_t lo, int64_t hi, int device,
                      int64_t* out);
void set_scan_server_off(bool off);
uint64_t scan_server_requests();
int launch_fill_prng(uint8_t* d_data, uint64_t stride, uint64_t stream_len, uint32_t nstreams, uint64_t seed,
                     uint64_t first_sid, void* stream);
// Grouped streaming handles: request r scans [lo, hi] of the `len` bytes at base + off.
struct ScanReq {
    uint64_t off;
    int64_t len, lo, hi;
};
int launch_scan_first_batch(const Algo& algo, const uint8_t* d_base, const ScanReq* d_reqs, uint32_t n, int64_t* d_out,
                            int device, void* stream, uint8_t* d_scratch = nullptr);  // scratch: as base's extent
size_t long_workspace_bytes(const Algo& algo, uint64_t len);
// Several long streams in one launch (segments of all streams scanned together, one
// resolving wave per stream).
size_t long_workspace_bytes_multi(const Algo& algo, const uint64_t* lens, uint32_t m);
int launch_split_long_multi(const Algo& algo, uint32_t m, const uint8_t* const* d_data, const uint64_t* lens,
                            uint64_t* const* d_cuts, const uint64_t* caps, uint64_t* const* d_counts, void* ws,
                            size_t ws_bytes, int device, void* stream);
int launch_split_long(const Algo& algo, const uint8_t* d_data, uint64_t len, uint64_t* d_cuts, uint64_t cuts_cap,
                      uint64_t* d_count, void* ws, size_t ws_bytes, int device, void* stream);

// ---- resumable content hashes (kcdc_hash.hip), for the batching writers
struct HashChain {       // one chunk's keyed BLAKE2 chain, in device memory (128 bytes)
    uint64_t h[8];       // the state (BLAKE2s: the low words)
    uint64_t src;        // the chunk's bytes (device address)
    uint64_t len;        // its length
    uint64_t next;       // message blocks compressed so far; ~0: not started (parameter and key blocks next)
    uint32_t out;        // digest slot
    uint32_t pad[9];
};
static_assert(sizeof(HashChain) == 128, "HashChain is 128 bytes");
// 1 BLAKE2b, 2 BLAKE2s (resumable), 3 another registered name (whole chunks), < 0 unknown; *out_len = digest bytes.
int hash_chain_kind(const char* name, uint32_t* out_len);
// Advance chains d_chains[d_active[0..n)] by at most max_blocks message blocks each; a chain that ends
// writes its digest to d_digests + out * digest_stride.  An entry with kChainNew set starts its chain
// from the record fresh[slot] (src, len, out; may be host-mapped pinned memory, as may d_active and
// d_digests).  Every chunk must start 16-byte aligned and be readable up to its length rounded up
// to 16.
constexpr uint32_t kChainNew = 0x80000000u;
int launch_hash_chains(const char* name, const uint8_t* key, uint32_t key_len, HashChain* d_chains,
                       const HashChain* fresh, const uint32_t* d_active, uint32_t nactive, uint64_t max_blocks,
                       uint8_t* d_digests, uint32_t digest_stride, void* stream);

}  // namespace kcdc
