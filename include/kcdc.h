/*
 * kcdc.h — C ABI of the MI355X-native content-defined-chunking splitter for
 * Kopia (library: kopia_amd/libkcdc.so, built for gfx950).
 *
 * This is the drop-in boundary for Kopia's `repo/splitter` package.  Every
 * entry point below names the reference interface it replaces
 * (paths relative to the kopia/kopia tree).  Plain pointers and sizes only;
 * no torch or HIP types appear in the signatures (streams are passed as
 * `void*` holding a hipStream_t, or NULL for the library's own stream).
 *
 * Semantics are bit-exact with the reference Go splitters: for any input bytes
 * and any slicing of them, the split points are the ones Kopia computes.
 *
 * Errors: functions returning `int` return KCDC_OK (0) or a negative KCDC_E*
 * code and set a thread-local message readable with kcdc_last_error().  There
 * is NO silent CPU fallback: if the GPU path cannot run, the call fails.
 */
#ifndef KCDC_H
#define KCDC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KCDC_OK 0
#define KCDC_ENOENT (-2)     /* unknown splitter name */
#define KCDC_EIO (-5)        /* HIP runtime / kernel error */
#define KCDC_ENOMEM (-12)
#define KCDC_EINVAL (-22)
#define KCDC_ENODEV (-19)    /* no usable gfx950 device */
#define KCDC_EOVERFLOW (-75) /* caller-provided cut capacity too small */
#define KCDC_EFBIG (-27)     /* chunk too long to encrypt (>= 1 GiB) */
#define KCDC_EBADMSG (-74)   /* sealed chunk failed authentication */

/* counts[i] value of every stream of a batch launch that could not complete on the
 * device (a wave gave up waiting in the work queue): the launch's cut lists are invalid.
 * The _host entry points return KCDC_EIO instead. */
#define KCDC_COUNT_FAILED UINT64_MAX

#define KCDC_KIND_FIXED 0
#define KCDC_KIND_BUZHASH 1
#define KCDC_KIND_RABINKARP 2

/* Parameters behind a registered name.
 * Reference: newBuzHash32SplitterFactory repo/splitter/splitter_buzhash32.go:73-86,
 * newRabinKarp64SplitterFactory splitter_rabinkarp64.go:73-83, Fixed splitter_fixed.go:33-37. */
typedef struct kcdc_algo_info {
    int32_t kind;      /* KCDC_KIND_* */
    int32_t pooled;    /* 1 if the reference wraps the factory in pooled() (splitter.go:51-73) */
    uint64_t avg;      /* average chunk size (FIXED: chunk length) */
    uint64_t min_size; /* avg/2 (FIXED: chunk length) */
    uint64_t max_size; /* 2*avg (FIXED: chunk length) == MaxSegmentSize() */
    uint64_t mask;     /* avg-1 (FIXED: 0) */
} kcdc_algo_info;

/* ------------------------------------------------------------ diagnostics */
const char* kcdc_last_error(void);
const char* kcdc_version(void);
/* Number of visible gfx950 devices (0 on a machine without one). */
int kcdc_device_count(void);

/* --------------------------------------------------------------- registry */
/* SupportedAlgorithms() — repo/splitter/splitter.go:32-42 (sorted names).
 * Writes up to `cap` name pointers (static storage) and returns the total count. */
int kcdc_supported_algorithms(const char** names, int cap);
/* DefaultAlgorithm — repo/splitter/splitter.go:89 ("DYNAMIC-4M-BUZHASH"). */
const char* kcdc_default_algorithm(void);
/* GetFactory(name) != nil — repo/splitter/splitter.go:84-86.  Returns KCDC_OK or KCDC_ENOENT. */
int kcdc_lookup(const char* name, kcdc_algo_info* info);
/* Factory().MaxSegmentSize() — splitter_buzhash32.go:69-71 / splitter_rabinkarp64.go:69-71 /
 * splitter_fixed.go:29-31.  Returns < 0 (KCDC_ENOENT) for unknown names. */
int64_t kcdc_max_segment_size(const char* name);
/* Name for a NON-registered parameterisation, mirroring the unexported factory
 * constructors the reference tests call directly: newBuzHash32SplitterFactory(avg)
 * (splitter_buzhash32.go:73), newRabinKarp64SplitterFactory(avg)
 * (splitter_rabinkarp64.go:73), Fixed(length) (splitter_fixed.go:33); see
 * repo/splitter/splitter_test.go:27-52.  `avg` must be a power of two >= 2 for
 * the rolling kinds (mask = avg-1), >= 1 for FIXED.  Returns an interned name
 * (static storage, never in kcdc_supported_algorithms) accepted by every
 * name-taking entry point, or NULL (KCDC_EINVAL). */
const char* kcdc_custom_algorithm(int32_t kind, uint64_t avg);
/* Upper bound on the number of chunks of a `stream_len`-byte stream (every chunk
 * but the last is >= min size): size cut arrays with it. */
uint64_t kcdc_cut_capacity(const char* name, uint64_t stream_len);

/* Rolling-hash constants as derived by the library (buzhash32 byte table,
 * Rabin-Karp polynomial and out/mod tables; rollinghash v4.0.0, go.mod:13).
 * Any pointer may be NULL.  Host-only: works without a GPU. */
int kcdc_tables(uint32_t* buzhash256, uint64_t* rabin_pol, uint64_t* rabin_out256, uint64_t* rabin_mod256);

/* ------------------------------------------------ streaming Splitter handle
 * Mirrors `type Splitter interface` (repo/splitter/splitter.go:20-29) and
 * `type Factory func() Splitter` (:45).  One handle per object writer; calls on
 * one handle must be serialised by the caller (objectWriter.mu,
 * repo/object/object_writer.go:114), handles are independent of each other.
 * `b` is borrowed for the call only (object_writer.go:121-129). */
typedef struct kcdc_splitter kcdc_splitter;
/* GetFactory(name)() — NULL on unknown name or no device (see kcdc_last_error). */
kcdc_splitter* kcdc_splitter_new(const char* name, int device);
/* NextSplitPoint(b) — returns n in 1..len (split AFTER byte n, n bytes consumed),
 * -1 if no split point (all consumed), or a KCDC_E* code (< -1) on failure. */
int64_t kcdc_splitter_next(kcdc_splitter* s, const uint8_t* b, size_t len);
/* MaxSegmentSize() */
int64_t kcdc_splitter_max_segment_size(const kcdc_splitter* s);
/* Reset() — splitter_buzhash32.go:20-24: back to the 64-zero window, count 0. */
void kcdc_splitter_reset(kcdc_splitter* s);
/* Close() — splitter_pool.go:18-22: Reset and return to the name's pool (pooled
 * names) or free.  The handle must not be used afterwards. */
void kcdc_splitter_close(kcdc_splitter* s);

/* ------------------------------------------------ grouped streaming handles
 * Kopia runs many object writers at once (snapshot/upload/upload.go:769-782),
 * each with its own Splitter fed 64 KiB slices (upload.go:394-407).  A group
 * batches the GPU work of all its handles' concurrent NextSplitPoint calls into
 * one launch: each call stages its slice into pinned memory from its own thread
 * and blocks until the group's launch returns its answer (same semantics and
 * results as kcdc_splitter_next on a private handle).  The group thread waits up
 * to `max_wait_us` for more calls (0: ship whatever is there) and takes at most
 * `max_batch` calls per launch (0: 256).  One name per group (a repository uses
 * one splitter).  Handles come from kcdc_group_splitter and are released with
 * kcdc_splitter_close.  kcdc_group_free may come first: the group then lives on
 * until its last handle is closed (no handle may be created after it). */
typedef struct kcdc_group kcdc_group;
kcdc_group* kcdc_group_new(const char* name, int device, uint32_t max_batch, uint32_t max_wait_us);
kcdc_splitter* kcdc_group_splitter(kcdc_group* g);
void kcdc_group_free(kcdc_group* g);

/* ------------------------------------------------ batching object writers
 * The writer-level form of the streaming handle: objectWriter.Write
 * (repo/object/object_writer.go:113-139) hands each 64 KiB slice (snapshot/upload/
 * upload.go:394-407) to kcdc_bw_write, which only copies it into pinned staging.  A batcher
 * thread ships every writer's staged bytes in one round (H2D, one batch-splitter launch over
 * all writers, cut lists back) once `round_bytes` are staged (0: 256 MiB) or `max_wait_us`
 * after the first staged byte (0: 2000).  Cut decisions therefore arrive later than the
 * bytes: kcdc_bw_cuts returns the FINAL cut offsets found so far (absolute offsets in the
 * object, strictly increasing, each a chunk end), and after kcdc_bw_finish (the object's
 * Close/Result: blocks until every byte is split) the remaining ones including the trailing
 * chunk's end.  The sequence is exactly the cuts of one NextSplitPoint pass over the whole
 * object, however it was sliced.  The writer must keep the bytes of its unflushed chunks
 * (objectWriter already buffers them in gather.WriteBuffer) and flush each chunk when its cut
 * arrives.  Calls on one writer are serialised by the caller; writers are independent.
 * kcdc_bw_write blocks while half a round of the writer's bytes is still unshipped.
 *
 * Devices: kcdc_bw_batcher_new_devices spreads the writers over a device set (`devices`, or
 * every device when NULL / ndev <= 0; an index may repeat, e.g. two logical devices on one
 * GPU).  Each device has its own round thread, streams and arenas; kcdc_bw_open assigns a writer
 * to the device with the least load (the bytes of its open writers, each counted as the larger
 * of its size hint and its bytes written: kcdc_bw_open_hint passes the object's expected size,
 * e.g. the file size the uploader knows, snapshot/upload/upload.go:769-782).  kcdc_bw_device
 * returns the writer's position in the device list.
 * Device memory: every open writer holds two arenas of about max_size + 4 x (round_bytes / 8 +
 * 4 MiB) bytes each (152 MiB at the defaults); kcdc_bw_open fails with KCDC_ENOMEM when the
 * device cannot hold them.
 * A freed writer's arenas are kept for the next kcdc_bw_open (hipMalloc/hipFree per object would
 * serialise on the device): at most as many pairs as writers were open at once, all given back
 * when a kcdc_bw_open would otherwise fail with KCDC_ENOMEM, and at kcdc_bw_batcher_free.
 * kcdc_bw_batcher_free ships what is staged, then fails every writer call still blocked in it
 * (KCDC_EINVAL) and waits for those calls to return; writers not freed before it stay valid for
 * kcdc_bw_free only.  A writer call that starts while or after kcdc_bw_batcher_free runs returns
 * KCDC_EINVAL without touching the freed batcher (its lifetime state is refcounted by its
 * writers), and kcdc_bw_free of such a writer waits until the batcher has let it go. */
typedef struct kcdc_bw_batcher kcdc_bw_batcher;
typedef struct kcdc_bw kcdc_bw;
kcdc_bw_batcher* kcdc_bw_batcher_new(const char* name, int device, uint64_t round_bytes, uint32_t max_wait_us);
kcdc_bw_batcher* kcdc_bw_batcher_new_devices(const char* name, const int* devices, int ndev, uint64_t round_bytes,
                                             uint32_t max_wait_us);
int kcdc_bw_batcher_devices(const kcdc_bw_batcher* b);  /* devices in the set */
void kcdc_bw_batcher_free(kcdc_bw_batcher* b);
kcdc_bw* kcdc_bw_open(kcdc_bw_batcher* b);        /* Factory() for one object */
kcdc_bw* kcdc_bw_open_hint(kcdc_bw_batcher* b, uint64_t size_hint);
int kcdc_bw_device(const kcdc_bw* w);             /* the writer's device (position in the list) */
int kcdc_bw_write(kcdc_bw* w, const uint8_t* p, size_t len);
int64_t kcdc_bw_cuts(kcdc_bw* w, uint64_t* out, uint64_t cap); /* final cuts taken (<= cap), or KCDC_E* */
int kcdc_bw_finish(kcdc_bw* w);
void kcdc_bw_free(kcdc_bw* w);
/* Content IDs (round 5): name every final chunk on the device, from the bytes the rounds already
 * hold, as the content manager does after the object writer flushes it
 * (repo/object/object_writer.go:186-227 -> repo/content/content_manager.go:812, hashData):
 * kcdc_bw_batcher_hash selects a registered hash name (kcdc_hash_algorithms; the repository's
 * hasher, hashing.go:51 defaults to BLAKE2B-256-128) and its HMAC secret, before the first writer
 * opens.  Then kcdc_bw_cuts_ids replaces kcdc_bw_cuts: it returns up to cap final cuts in order, each
 * with its chunk's digest (kcdc_hash_size bytes at ids + i * id_stride), as soon as the digests of
 * every chunk up to it are known; kcdc_bw_finish also waits for the last chunk's digest.  BLAKE2
 * names hash in slices of 256 KiB per chunk per step (a chunk is one chain of compressions), the
 * others whole chunks per step, on a hash thread of their own.  Device memory: an ID ring of
 * max(64 x round_bytes, 1 GiB) per device holds the chunks until they are named (a chunk is one
 * dependent chain, so the naming rate grows with the chunks in flight).  FIXED names: KCDC_EINVAL
 * (their writers stage no bytes on the device). */
int kcdc_bw_batcher_hash(kcdc_bw_batcher* b, const char* hash_name, const uint8_t* key, uint32_t key_len);
int64_t kcdc_bw_cuts_ids(kcdc_bw* w, uint64_t* cuts, uint8_t* ids, uint32_t id_stride, uint64_t cap);
int64_t kcdc_bw_rounds(const kcdc_bw_batcher* b); /* rounds shipped so far (test hook) */
/* Observability (summed over the batcher's devices; the span and busy seconds are the largest
 * device's): out[0..n) = rounds, bytes shipped, seconds the round thread spent building and
 * issuing rounds, seconds it waited for the device, then the device seconds of the rounds' gathers
 * (new bytes over PCIe into the writers' arenas) and of their splits (metadata in, splitter
 * launch, cut lists out), from HIP events, then the device span of all rounds and the seconds of
 * it in which a gather or a split ran, then the round thread's seconds per phase (collecting the
 * writers' blocks, placing them in the arenas, issuing the gather, waiting for the previous round,
 * issuing the split), then the round thread's seconds waiting for a round's worth of staged bytes,
 * and the writers' seconds (summed over writers) blocked on their staging cap and getting a pinned
 * staging block, then the pinned blocks allocated because the pool was empty and the round
 * thread's seconds acquiring the batcher's mutex to apply a finished round, then (content IDs)
 * the chunks named, the hash steps issued and their device seconds, the round thread's seconds
 * waiting for ID ring space, the hash thread's seconds with no step to issue, and the chains
 * advanced summed over steps.  Returns 24. */
int kcdc_bw_stats(kcdc_bw_batcher* b, double* out, int n);

/* ------------------------------------------------------ batch (hot path)
 * Split `nstreams` independent streams in one launch; every stream starts from
 * a fresh splitter (the pool's Reset-on-Close, splitter_pool.go:18-22).
 * Output for stream i: counts[i] chunk END offsets written to
 * cuts[cut_base[i] .. cut_base[i]+counts[i]), strictly increasing, the last one
 * equal to lens[i] (the trailing chunk `Result()` flushes,
 * repo/object/object_writer.go:264-277).  An empty stream yields 0 entries.
 * Capacity for stream i is cut_base[i+1]-cut_base[i] (last: `cuts_cap`-cut_base[i]);
 * size it with kcdc_cut_capacity().  counts[i] always receives the TRUE number of
 * chunks; entries beyond the capacity are not written, so counts[i] > capacity
 * signals overflow (the _host variant returns KCDC_EOVERFLOW).
 *
 * _device: every pointer (the array of stream pointers, lens, cuts, cut_base,
 * counts) is device memory on the current device; the call is asynchronous on
 * `hip_stream` (NULL = legacy default stream) except for error checking of
 * the launch.  A launch that fails on the device sets every counts[i] to
 * KCDC_COUNT_FAILED (no partial results are ever reported as complete).  Stream bytes may have any alignment.  Each launch takes one of 64
 * per-device queue workspaces in turn; a launch that reuses a workspace still in
 * use by another stream waits for it (an event), so any number may be in flight. */
int kcdc_split_batch_device(const char* name, const uint8_t* const* d_ptrs, const uint64_t* d_lens,
                            uint32_t nstreams, uint64_t* d_cuts, uint64_t cuts_cap, const uint64_t* d_cut_base,
                            uint64_t* d_counts, void* hip_stream);

/* _host: host buffers in, host cut lists out.  Streams are copied H2D in groups
 * of <= 1 GiB (the HIP runtime stages pageable memory; buffers the caller
 * allocated pinned are DMA'd directly), each group split like
 * kcdc_split_files_device (large streams through the long-stream path), and the
 * cut lists copied back.  Synchronous, PCIe-bound.  This is the
 * path the Go cgo shim calls. */
int kcdc_split_batch_host(const char* name, const uint8_t* const* h_ptrs, const uint64_t* lens, uint32_t nstreams,
                          uint64_t* cuts, uint64_t cuts_cap, const uint64_t* cut_base, uint64_t* counts, int device);
/* The same over a device set (`devices`, repeats allowed; NULL / ndev <= 0: every device): the
 * streams are spread by bytes with kcdc_lpt_assign and each device splits its share from a host
 * thread of its own (no collectives: SURVEY.md §8e).  Same output contract as one device. */
int kcdc_split_batch_host_devices(const char* name, const int* devices, int ndev, const uint8_t* const* h_ptrs,
                                  const uint64_t* lens, uint32_t nstreams, uint64_t* cuts, uint64_t cuts_cap,
                                  const uint64_t* cut_base, uint64_t* counts);
/* Longest-processing-time-first assignment by bytes (largest stream first, each to the least
 * loaded of `ndev` devices, ties to the lower index): dev_of[i] = position of stream i's device. */
int kcdc_lpt_assign(const uint64_t* lens, uint32_t nstreams, uint32_t ndev, uint32_t* dev_of);

/* ------------------------------------------- one long stream, tiled (config 3)
 * Exact intra-stream parallel CDC of a single device-resident stream: candidate
 * scan over all tiles in parallel, then chunk resolution on the device.  The
 * cut set is identical to one sequential pass (no Concatenate seams; cf.
 * snapshot/upload/upload.go:166-209, repo/object/object_manager.go:102-152).
 * `workspace` must hold kcdc_long_workspace_bytes(name, len) bytes of device
 * memory.  d_count receives the number of cuts written to d_cuts. */
size_t kcdc_long_workspace_bytes(const char* name, uint64_t len);
int kcdc_split_long_device(const char* name, const uint8_t* d_data, uint64_t len, uint64_t* d_cuts, uint64_t cuts_cap,
                           uint64_t* d_count, void* workspace, size_t workspace_bytes, void* hip_stream);

/* ------------------------------------------- many streams of any sizes (config 5)
 * Splits n streams of arbitrary lengths (e.g. the files of one upload,
 * snapshot/upload/upload.go:769-782) with the same output contract as
 * kcdc_split_batch_device, routing each stream to the path that finishes it
 * soonest: streams that one wavefront would still be scanning after the rest
 * of the batch is done (the largest ones, >= 1 MiB) go through the long-stream
 * path, the others through one batch launch.  Boundaries are identical either
 * way.  h_dptrs (device addresses), h_lens and h_cut_base are HOST arrays;
 * d_cuts and d_counts are device memory.  Asynchronous on `hip_stream`
 * (stream-ordered allocations for scratch). */
int kcdc_split_files_device(const char* name, const uint8_t* const* h_dptrs, const uint64_t* h_lens, uint32_t n,
                            uint64_t* d_cuts, uint64_t cuts_cap, const uint64_t* h_cut_base, uint64_t* d_counts,
                            void* hip_stream);

/* ------------------------------------------------- synthetic input (bench)
 * Fill `nstreams` device streams of `stream_len` bytes each, laid out at
 * d_data + i*stride, with the counter-PRNG bytes of stream id (first_sid + i)
 * (bytes are a pure function of (seed, sid, offset); BASELINE.json configs 2-5). */
int kcdc_fill_prng(uint8_t* d_data, uint64_t stride, uint64_t stream_len, uint32_t nstreams, uint64_t seed,
                   uint64_t first_sid, void* hip_stream);

/* rand.New(rand.NewSource(seed)).Read(out[:n]) of Go math/rand: the input of
 * `kopia benchmark splitter` (cli/command_benchmark_splitters.go:66-75, one Rand
 * read block after block, so consecutive blocks are one continuous read).
 * Host-only (no GPU needed). */
int kcdc_gorand_read(int64_t seed, uint8_t* out, uint64_t n);

/* ------------------------------------------------------------- content hashes
 * The content hash Kopia computes for every chunk the splitter cuts, for many chunks of
 * device-resident bytes (repo/content/content_manager.go:812 -> repo/hashing/hashing.go:55-103).
 * Every registered name (hashing.SupportedAlgorithms(), sorted):
 *   "BLAKE2B-256", "BLAKE2B-256-128" (the default, hashing.go:51), "BLAKE2S-128", "BLAKE2S-256"
 *     keyed BLAKE2 (blake_hashes.go:8-13, truncatedKeyedHashFuncFactory);
 *   "BLAKE3-256", "BLAKE3-256-128": blake3.NewKeyed(key), key = the secret's first 32 bytes, or
 *     blake3.DeriveKey("kopia blake3 derived key v1", secret) for a shorter secret
 *     (blake3_hashes.go:10-27);
 *   "HMAC-SHA224", "HMAC-SHA256", "HMAC-SHA256-128", "HMAC-SHA3-224", "HMAC-SHA3-256":
 *     hmac.New(sha*, secret), truncated (sha_hashes.go:9-15; any key length).
 * kcdc_hash_algorithms: fills names[0..cap) and returns the count.
 * kcdc_hash_size: output bytes per chunk (16, 28 or 32), or KCDC_ENOENT.
 * kcdc_hash_chunks_device: chunk i is bytes [d_offsets[i], d_offsets[i] + d_lens[i]) of
 *   d_data (any alignment); its hash goes to d_out + i * out_stride (out_stride >= the hash
 *   size, a multiple of 4).  key: the repository's HMAC secret (<= 64 bytes for BLAKE2B,
 *   <= 32 for BLAKE2S; BLAKE2S-128 needs one, as blake2s.New128 does).  d_order: optional
 *   processing order (e.g. chunk indices by descending length: a wave runs until its
 *   longest chunk is done), NULL = as given.  Asynchronous on hip_stream. */
int kcdc_hash_algorithms(const char** names, int cap);
int kcdc_hash_size(const char* hash_name);
int kcdc_hash_chunks_device(const char* hash_name, const uint8_t* d_data, const uint64_t* d_offsets,
                            const uint64_t* d_lens, const uint32_t* d_order, uint32_t nchunks, const uint8_t* key,
                            uint32_t key_len, uint8_t* d_out, uint32_t out_stride, void* hip_stream);

/* ------------------------------------------------------------- content encryption
 * Side channels: the AES-256-GCM kernels look up AES T-tables and GHASH tables in LDS with key- and
 * data-dependent indices (gfx950 has no AES or carry-less-multiply instructions), so they are not
 * constant-time, unlike Go's AES-NI path; use them on a single-tenant GPU.  ChaCha20-Poly1305 has no
 * table lookups.  
 * Kopia's two encryptors, AES256-GCM-HMAC-SHA256 (the default; repo/encryption/
 * aes256_gcm_hmac_sha256_encryptor.go:24-72) and CHACHA20-POLY1305-HMAC-SHA256
 * (chacha20_poly1305_hmac_sha256_encryptor.go: Encrypt/Decrypt/Overhead, 24-80; both through
 * aead_helpers.go:12-75), for many chunks per call, selected by `algorithm`:
 *   key_i  = HMAC-SHA256(secret, id_i)      id_i = the content ID the Encryptor is given; the content
 *            manager passes the last 16 bytes of the content hash (getPackedContentIV,
 *            repo/content/content_manager_lock_free.go:178-182)
 *   sealed = nonce_i(12) || AEAD(key_i, nonce_i, plaintext, aad = id_i)
 *            AEAD = AES-256-GCM (NIST SP 800-38D) or ChaCha20-Poly1305 (RFC 8439); 16-byte tag
 * secret: the repository's derived key, HKDF-SHA256(masterKey, "encryption", "", 32)
 *   (deriveKey, repo/encryption/encryption.go:80-92), 1..64 bytes.
 * kcdc_encryption_algorithms / kcdc_encryption_overhead (28): the registry (Register, encryption.go:65).
 * kcdc_crypt_workspace_size(n): bytes of device scratch a call over n chunks needs, for either
 *   algorithm (~9 KiB per chunk: its key and a table of powers of r, or of H for GCM).
 * kcdc_encrypt_chunks_device: plaintext i = [d_offsets[i], +d_lens[i]) of d_data (any
 *   alignment, < 1 GiB); d_nonces: 12 bytes per chunk (the reference draws them from
 *   crypto/rand; the caller does here); the sealed chunk (d_lens[i] + 28 bytes) is written at
 *   d_out + d_out_offsets[i] (a multiple of 4).  d_status[i]: 0, or KCDC_EFBIG (too long).
 * kcdc_decrypt_chunks_device: sealed chunk i = [d_offsets[i], +d_sealed_lens[i]) of
 *   d_sealed; its plaintext (d_sealed_lens[i] - 28 bytes) goes to d_out + d_out_offsets[i]
 *   (a multiple of 4; up to 3 zero bytes of padding after it are written too).
 *   d_status[i]: 0, KCDC_EBADMSG (authentication failed: aeadOpenPrefixedWithNonce's "unable to
 *   decrypt content"; the plaintext slot holds unauthenticated bytes), KCDC_EINVAL (shorter than
 *   28 bytes: "ciphertext too short") or KCDC_EFBIG.
 * d_ivs: iv_len (1..64) bytes per chunk at d_ivs + i * iv_stride: the content IDs (e.g. the
 * hash output of kcdc_hash_chunks_device + hash size - 16, iv_len 16).  Asynchronous on hip_stream; d_work must stay
 * allocated until the work finishes. */
int kcdc_encryption_algorithms(const char** names, int cap);
int kcdc_encryption_overhead(const char* algorithm);
uint64_t kcdc_crypt_workspace_size(uint32_t nchunks);
int kcdc_encrypt_chunks_device(const char* algorithm, const uint8_t* secret, uint32_t secret_len, const uint8_t* d_data,
                               const uint64_t* d_offsets, const uint64_t* d_lens, uint32_t nchunks,
                               const uint8_t* d_ivs, uint32_t iv_len, uint32_t iv_stride, const uint8_t* d_nonces,
                               uint8_t* d_out,
                               const uint64_t* d_out_offsets, int32_t* d_status, void* d_work, uint64_t work_bytes,
                               void* hip_stream);
int kcdc_decrypt_chunks_device(const char* algorithm, const uint8_t* secret, uint32_t secret_len,
                               const uint8_t* d_sealed, const uint64_t* d_offsets, const uint64_t* d_sealed_lens,
                               uint32_t nchunks, const uint8_t* d_ivs, uint32_t iv_len, uint32_t iv_stride,
                               uint8_t* d_out,
                               const uint64_t* d_out_offsets, int32_t* d_status, void* d_work, uint64_t work_bytes,
                               void* hip_stream);

/* ------------------------------------------------------------- content compression
 * Kopia's compressors (header IDs compression_ids.go:8-30) for many chunks per call, with the
 * content manager's keep-or-drop rule (maybeCompressAndEncryptDataForPacking,
 * repo/content/content_manager_lock_free.go:42-73):
 *   out_i = BE32(header ID) || the compressed stream of chunk i
 *   id_i  = header ID if len(out_i) < len(chunk i), else 0 (NoCompression: store chunk i as is)
 * Streams: deflate-* raw DEFLATE (RFC 1951; compressor_deflate.go:14-62), gzip* / pgzip* the same
 * stream in an RFC 1952 member with its CRC-32 and ISIZE (compressor_gzip.go:15-17,
 * compressor_pgzip.go:16-18), s2-* the S2 framing format with CRC-32C-checked chunks of Snappy
 * elements (compressor_s2.go:20-23), zstd* one RFC 8878 frame (compressor_zstd.go:15-18).  The
 * reference's readers (flate/gzip/pgzip/s2/zstd NewReader) read out_i after its 4 header bytes;
 * the bytes are this encoder's, not klauspost/compress's.
 * kcdc_compression_algorithms: the names encoded on the device; kcdc_compression_header_id: a
 *   name's header ID (or a negative error).
 * kcdc_compress_bound(len): the largest out_i for a chunk of len bytes (24 + len + 5 per 512 bytes).
 * kcdc_compress_workspace_size(total, n): device scratch for n chunks of `total` bytes in all
 *   (~1.13 bytes per input byte).
 * kcdc_compress_chunks_device: chunk i = [d_offsets[i], +d_lens[i]) of d_data (any alignment);
 *   out_i goes to d_out + d_out_offsets[i] (room for kcdc_compress_bound bytes), its length to
 *   d_out_lens[i] and id_i to d_header_ids[i].  A workspace too small for the chunks' spans
 *   leaves every d_out_lens[i] = 0.  Asynchronous on hip_stream. */
int kcdc_compression_algorithms(const char** names, int cap);
int64_t kcdc_compression_header_id(const char* algorithm);
uint64_t kcdc_compress_bound(uint64_t len);
uint64_t kcdc_compress_workspace_size(uint64_t total_bytes, uint32_t nchunks);
int kcdc_compress_chunks_device(const char* algorithm, const uint8_t* d_data, const uint64_t* d_offsets,
                                const uint64_t* d_lens, uint32_t nchunks, uint8_t* d_out,
                                const uint64_t* d_out_offsets, uint64_t* d_out_lens, uint32_t* d_header_ids,
                                void* d_work, uint64_t work_bytes, void* hip_stream);

/* ------------------------------------------------------------- testing
 * Hooks for the library's own tests (not part of the splitter surface).
 * kcdc_test_set: process-wide knobs read by every later batch launch.
 *   KCDC_TEST_SPIN_CAP    polls with no stream finishing before a waiting wave gives up, the
 *                         current poll included (0: default, ~seconds; 1: at the first
 *                         unready poll)
 *   KCDC_TEST_NO_STEAL    1: waves never requeue the streams of workgroups that have not started
 *   KCDC_TEST_FORCE_ERROR 1: every batch launch reports failure (KCDC_COUNT_FAILED)
 *   KCDC_TEST_HASH_LANES  lanes per chunk of kcdc_hash_chunks_device: 0 auto (4 up to 2^20
 *                         chunks, else 1), 1 or 4
 *   KCDC_TEST_NO_SERVER   1: private streaming handles launch one scan per call instead of using
 *                         the device's resident scan server
 *   KCDC_TEST_NO_HELP     1: batch launches without intra-region help (each region is scanned by
 *                         the wave that owns its stream only); 2: help on whatever the average
 *                         (0, the default: help for averages of 1 MiB and up, and for Rabin-Karp
 *                         launches with fewer streams than waves)
 *   KCDC_TEST_ID_RING     bytes of the writers' content-ID ring for batchers created from now on
 *                         (0: the default; small values exercise wrap-around and backpressure)
 *   KCDC_TEST_LANE_CAP    buzhash batch launches: bytes per lane segment (a tile is 64 of them),
 *                         a power of two in [256, 4096]; 0: the default (avg / 256 within
 *                         [256, 2048]).  Other tile geometries for the same cuts.
 * kcdc_test_occupy: occupy `nwg` CUs (one workgroup with all of the CU's LDS each) for
 * `usec` microseconds on `hip_stream`, e.g. to run a batch beside a kernel that holds CUs.
 * kcdc_test_queue_stat: after the last pipelined batch launch has finished (synchronise
 * first), read one word of its queue header: KCDC_TEST_STAT_GIVEUPS (waves that gave up
 * waiting), KCDC_TEST_STAT_DONE (streams finished), KCDC_TEST_STAT_STEALS (requeued
 * workgroups), KCDC_TEST_STAT_HELPS (tiles scanned by waves that helped another wave's region),
 * KCDC_TEST_STAT_TICKETS / KCDC_TEST_STAT_ENTRIES (the ring's ticket and entry counters) and
 * KCDC_TEST_STAT_WAVES (the launch's waves).  Every wave exits holding one ticket and every
 * reserved entry is written, so TICKETS - ENTRIES is WAVES (WAVES - 1 when the last stream's
 * final entry is a tombstone nobody waited for).  Synchronous copy; returns the word, or a
 * negative KCDC_E* code. */
#define KCDC_TEST_SPIN_CAP 1
#define KCDC_TEST_NO_STEAL 2
#define KCDC_TEST_FORCE_ERROR 3
#define KCDC_TEST_HASH_LANES 4
#define KCDC_TEST_NO_SERVER 5
#define KCDC_TEST_NO_HELP 6
#define KCDC_TEST_ID_RING 7
#define KCDC_TEST_LANE_CAP 8
int kcdc_test_set(int32_t key, int64_t value);
int kcdc_test_occupy(uint32_t nwg, uint32_t usec, void* hip_stream);
#define KCDC_TEST_STAT_GIVEUPS 1
#define KCDC_TEST_STAT_DONE 2
#define KCDC_TEST_STAT_STEALS 3
#define KCDC_TEST_STAT_HELPS 4
#define KCDC_TEST_STAT_TICKETS 10
#define KCDC_TEST_STAT_ENTRIES 11
#define KCDC_TEST_STAT_WAVES 12
int64_t kcdc_test_queue_stat(int32_t key);
/* Test hook: copy bytes [off, off + n) of the last pipelined launch's queue workspace (queue
 * header, stream ring, help slots) to host memory at dst; 0 or a negative error. */
int kcdc_test_ws_copy(void* dst, uint64_t off, uint64_t n);
/* Requests the resident scan server has answered in this process (private streaming handles use
 * it while exactly one private handle is open). */
int64_t kcdc_test_server_requests(void);

#ifdef __cplusplus
}
#endif
#endif /* KCDC_H */
