// datafile_hip.hip -- f3: record-boundary discovery for 0-db datafile images
// resident in HBM, and the device-resident integrity scan built on it
// (tools/integrity-check over a whole store, integrity-check.c:59-105).
//
// The reference finds records with a serial chain: each entry header gives
// the next offset, pos' = pos + 18 + idlength + datalength
// (integrity-check.c:59-69, data.c:306-311; host form: datafile.c).  A GPU
// cannot follow one chain fast (one dependent HBM round trip per record), so
// every file is cut into chunks of C bytes (default 8 MiB) and the chain is
// discovered speculatively and stitched exactly:
//
//   A1 search  (one workgroup of 4 waves per chunk): the first position
//              p >= chunk start that looks like an entry header -- top byte
//              of datalength 0 (the writer caps payloads at 8 MiB, data.h:6),
//              flags <= 3 (data.h:47-51) -- and whose successor
//              q = p + 18 + idlength + datalength names p as its `previous`
//              entry (data_insert, data.c:601), or ends the file.  Each wave
//              takes 8 KiB blocks (64 lanes x 16 positions x 8, all loads in
//              flight), one zero-byte test per 4 positions; a random position
//              passes the filter with p ~ 2^-14 and the back-pointer check
//              with p ~ 2^-32.
//   A2 walk    (one thread per chunk, 64 chains in flight per wave): follow
//              the chain from that candidate to the first header at or past
//              the chunk end (its "exit"), counting records, stopping on the
//              serial walk's terminal conditions (clean EOF, short header,
//              short payload).
//   B  stitch  (one thread per file): chunk 0 starts at offset 28, exactly
//              where the reference starts.  Chunk c is accepted when its
//              speculative start equals the true exit of chunk c-1; a chunk
//              that no record starts in is skipped; otherwise (a false
//              candidate, or a true header the filter rejected: a file not
//              written by zdbd, a rewritten `previous` chain) the chunk is
//              re-walked serially from the true exit.  So the result is the
//              serial walk's, whatever the filter decides -- the filter only
//              decides how much is parallel.
//   B2 prefix  record counts of the files -> global record index base.
//   C  emit    (one thread per chunk): re-follow the accepted chain and write
//              the descriptors in file order.
//
// The integrity scan then verifies the emitted descriptors with the batched
// checksum kernel (zdb_crc32_verify_device).  Bytes per record: ~3 header
// reads of a few bytes (A2, C) + the search windows (on average the
// remainder of the record straddling each chunk start).

#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>

#include <hip/hip_runtime.h>

#include "zdb_crc32.h"
#include "zdb_datafile.h"

extern "C" void zdbcrc_internal_mark_hip(void); // crc32_hip.hip (not exported)

namespace {

constexpr uint64_t NONE = ~0ull;
constexpr int32_t ST_CONTINUE = -1;
// 8 MiB chunks: C4 (64 x 256 MiB files of C3 payloads) walks in 0.83 ms
// against 0.91 (4 MiB), 1.28 (2 MiB) and 1.24 ms (16 MiB) --
// profiles/r2/walk_probe.jsonl; smaller chunks search more, larger ones
// follow longer chains
constexpr uint32_t DEFAULT_LG_CHUNK = 23;
constexpr uint32_t WALK_T = 256;
constexpr int SU = 8; // search: KiB per wave iteration

// little-endian u32 at any byte address: two aligned dword loads + one
// v_alignbyte (reads up to 7 bytes past p; images are readable 16 bytes past
// their end, as for the checksum kernel)
__device__ __forceinline__ uint32_t ld_le32(const uint8_t *p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t *q = reinterpret_cast<const uint32_t *>(a & ~uintptr_t(3));
    return __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(a & 3));
}

// the fields of the entry header at pos the walk needs (data.h:56-65):
// idlength (byte 0), datalength (1..4), integrity (9..12).  Five aligned
// dword loads issued together -- one memory round trip per record (reads up
// to pos + 20, within the 16 readable bytes past the file when pos + 4 <= len)
struct Hdr {
    uint32_t idl, L, integ;
};
__device__ __forceinline__ Hdr load_hdr(const uint8_t *f, uint64_t len, uint64_t pos) {
    if (pos + 4 <= len) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(f + pos);
        const uint32_t *q = reinterpret_cast<const uint32_t *>(a & ~uintptr_t(3));
        const uint32_t sh = (uint32_t)(a & 3);
        const uint32_t q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3], q4 = q[4];
        const uint32_t w0 = __builtin_amdgcn_alignbyte(q1, q0, sh), w1 = __builtin_amdgcn_alignbyte(q2, q1, sh);
        const uint32_t w2 = __builtin_amdgcn_alignbyte(q3, q2, sh), w3 = __builtin_amdgcn_alignbyte(q4, q3, sh);
        return Hdr{w0 & 0xFFu, (w0 >> 8) | (w1 << 24), (w2 >> 8) | (w3 << 24)};
    }
    return Hdr{f[pos], 0u, 0u}; // no whole header fits: the walk stops on SHORT_HEADER
}

// one record of the serial walk at pos (datafile.c zdb_datafile_walk):
// SHORT_HEADER -> not a record; SHORT_PAYLOAD -> a record that ends the walk
__device__ __forceinline__ int32_t hop(const uint8_t *f, uint64_t len, uint64_t pos, uint64_t &next,
                                       uint32_t &L, Hdr &h) {
    h = load_hdr(f, len, pos);
    const uint64_t hlen = ZDB_ENTRY_HEADER_SIZE + (uint64_t)h.idl;
    if (pos + hlen > len)
        return ZDB_WALK_SHORT_HEADER;
    L = h.L;
    next = pos + hlen;
    if (L) {
        if (next + L > len)
            return ZDB_WALK_SHORT_PAYLOAD;
        next += L;
    }
    return ST_CONTINUE;
}

// what a walked record turns into: image offsets of header and payload, and
// the checksum descriptor (length and expected crc are 0 for the records the
// integrity check skips: datalength 0, integrity-check.c:81-82, and a
// payload cut by the end of the file)
struct RecSlot {
    uint32_t pos;    // file-relative header offset (datafiles are < 4 GiB)
    uint32_t len;    // payload length to checksum
    uint32_t expect; // stored integrity
    uint32_t hlen;   // 18 + idlength
};

enum WalkMode { COUNT = 0, SPEC = 1, EMIT = 2 };

// follow the chain from pos while pos < cend.  SPEC keeps the first kcap
// records in the chunk's slots; EMIT writes the final descriptors at idx..
template <int MODE>
__device__ __forceinline__ void walk_chain(const uint8_t *f, uint64_t len, uint64_t pos, uint64_t cend,
                                           uint32_t &count, uint64_t &exit, int32_t &st, RecSlot *slots,
                                           uint32_t kcap, uint64_t foff, uint64_t idx, uint64_t capacity,
                                           uint64_t *__restrict__ entry_off, uint64_t *__restrict__ poff,
                                           uint32_t *__restrict__ plen, uint32_t *__restrict__ expect) {
    count = 0;
    st = ST_CONTINUE;
    while (pos < cend) {
        if (pos >= len) { // clean end of file (pos == len)
            st = ZDB_WALK_OK;
            break;
        }
        uint64_t next = 0;
        uint32_t L = 0;
        Hdr h;
        const int32_t s = hop(f, len, pos, next, L, h);
        if (s == ZDB_WALK_SHORT_HEADER) {
            st = s;
            break;
        }
        if (MODE != COUNT) {
            const bool full = s == ST_CONTINUE && L > 0; // payload present and non-empty
            const uint32_t hlen = ZDB_ENTRY_HEADER_SIZE + h.idl;
            const uint32_t ex = full ? h.integ : 0u;
            if (MODE == SPEC && count < kcap) {
                slots[count] = RecSlot{(uint32_t)pos, full ? L : 0u, ex, hlen};
            } else if (MODE == EMIT && idx < capacity) {
                entry_off[idx] = foff + pos;
                poff[idx] = foff + pos + hlen;
                plen[idx] = full ? L : 0u;
                expect[idx] = ex;
            }
        }
        idx++;
        count++;
        if (s == ZDB_WALK_SHORT_PAYLOAD) {
            st = s;
            break;
        }
        pos = next;
    }
    if (st == ST_CONTINUE && pos >= len)
        st = ZDB_WALK_OK;
    exit = pos;
}

// is there an entry header at p whose chain is consistent one step ahead?
__device__ __forceinline__ bool plausible_successor(const uint8_t *f, uint64_t len, uint64_t p, uint32_t idl,
                                                    uint32_t L) {
    const uint64_t q = p + ZDB_ENTRY_HEADER_SIZE + idl + L;
    if (q == len)
        return true;
    if (q + ZDB_ENTRY_HEADER_SIZE > len)
        return false;
    return ld_le32(f + q + 5) == (uint32_t)p; // q's `previous` (data.h:59)
}

struct FileTab {
    const uint8_t *image;
    const uint64_t *file_off;
    const uint64_t *file_len;
    uint32_t nfiles;
    uint32_t cpf; // chunks per file (grid)
    uint32_t lg;  // log2 chunk bytes
};

// candidate positions among the 16 starting at a 16-byte block whose 32
// bytes are d[0..7]: byte p+4 (top byte of datalength) is 0 and byte p+13
// (flags) is <= 3.  One zero-byte test covers 4 positions: bit 8r+7 of z[j]
// is set when position 4j+r qualifies (the test has no false negatives;
// false positives only cost a back-pointer check).
__device__ __forceinline__ uint32_t haszero(uint32_t x) { return (x - 0x01010101u) & ~x & 0x80808080u; }

__device__ __forceinline__ void candidates(const uint32_t (&d)[8], uint32_t (&z)[4]) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t fl = __builtin_amdgcn_alignbyte(d[j + 4], d[j + 3], 1u); // bytes 4j+13 .. 4j+16
        z[j] = haszero(d[j + 1]) & haszero(fl & 0xFCFCFCFCu);
    }
}

// A1: speculative start of every chunk (one workgroup of NWS waves per chunk:
// the waves take interleaved SU-KiB blocks, so a chunk that starts inside a
// 1 MiB payload is searched NWS blocks at a time)
__global__ __launch_bounds__(WALK_T) void walk_search_kernel(FileTab t, uint64_t *__restrict__ s_start,
                                                             int32_t *__restrict__ s_status) {
    constexpr uint32_t NWS = WALK_T / 64;
    constexpr uint64_t SB = 1024u * SU; // bytes per wave block
    __shared__ unsigned long long best;
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    const uint64_t w = blockIdx.x;
    const uint32_t fi = (uint32_t)(w / t.cpf), c = (uint32_t)(w % t.cpf);
    const uint64_t len = t.file_len[fi];
    const uint8_t *f = t.image + t.file_off[fi];
    const uint64_t C = 1ull << t.lg, c0 = (uint64_t)c * C;
    if (c == 0) {
        if (threadIdx.x == 0) {
            // data_descriptor_load / _validate (data.c:177-209): 28-byte
            // header, magic "DAT0", version 3
            const bool bad = len < ZDB_DATA_HEADER_SIZE || f[0] != 'D' || f[1] != 'A' || f[2] != 'T' ||
                             f[3] != '0' || ld_le32(f + 4) != ZDB_DATAFILE_VERSION;
            s_start[w] = bad ? NONE : (uint64_t)ZDB_DATA_HEADER_SIZE;
            s_status[w] = bad ? ZDB_WALK_BAD_DESCRIPTOR : ST_CONTINUE;
        }
        return;
    }
    if (c0 >= len || len < ZDB_ENTRY_HEADER_SIZE) {
        if (threadIdx.x == 0) {
            s_start[w] = NONE;
            s_status[w] = ST_CONTINUE;
        }
        return;
    }
    // positions p in [c0, c0 + C) with a whole 18-byte header in the file
    const uint64_t lim = (c0 + C < len - (ZDB_ENTRY_HEADER_SIZE - 1)) ? c0 + C : len - (ZDB_ENTRY_HEADER_SIZE - 1);
    if (threadIdx.x == 0)
        best = NONE;
    __syncthreads();
    for (uint64_t r0 = c0;; r0 += NWS * SB) {
        const uint64_t b = r0 + wid * SB;
        uint64_t found = NONE;
        if (b < lim) {
            uint4 a0[SU], a1[SU];
#pragma unroll
            for (int u = 0; u < SU; u++) { // every load of the block in flight
                const uint64_t p0 = b + 1024u * u + 16u * lane; // 16-byte aligned (c0 is a multiple of C)
                if (p0 < lim) {
                    a0[u] = *reinterpret_cast<const uint4 *>(f + p0);
                    a1[u] = *reinterpret_cast<const uint4 *>(f + p0 + 16);
                } else {
                    a0[u] = a1[u] = make_uint4(~0u, ~0u, ~0u, ~0u); // no candidate
                }
            }
#pragma unroll
            for (int u = 0; u < SU; u++) {
                const uint64_t p0 = b + 1024u * u + 16u * lane;
                const uint32_t d[8] = {a0[u].x, a0[u].y, a0[u].z, a0[u].w, a1[u].x, a1[u].y, a1[u].z, a1[u].w};
                uint32_t z[4];
                candidates(d, z);
                uint64_t hit = 0;
                if (z[0] | z[1] | z[2] | z[3]) { // rare: confirm through the successor's back-pointer
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        uint32_t m = z[j];
                        while (m && found == NONE) {
                            const uint32_t r = (uint32_t)__builtin_ctz(m) >> 3;
                            m &= ~(0xFFu << (8 * r));
                            const uint64_t p = p0 + 4u * j + r;
                            if (p < lim) {
                                const Hdr h = load_hdr(f, len, p);
                                if (plausible_successor(f, len, p, h.idl, h.L))
                                    found = p;
                            }
                        }
                    }
                }
                hit = __ballot(found != NONE);
                if (hit) { // lanes hold increasing addresses: the lowest lane has the block's first candidate
                    const uint32_t l = (uint32_t)__builtin_ctzll(hit);
                    found = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(found >> 32), l) << 32) |
                            __builtin_amdgcn_readlane((uint32_t)found, l);
                    break;
                }
            }
            if (found != NONE && lane == 0)
                atomicMin(&best, (unsigned long long)found);
        }
        __syncthreads();
        const uint64_t bst = best;
        __syncthreads();
        if (bst != NONE || r0 + NWS * SB >= lim) { // first block with a hit found, or the chunk is done
            if (threadIdx.x == 0) {
                s_start[w] = bst;
                s_status[w] = ST_CONTINUE;
            }
            return;
        }
    }
}

// A2: speculative chain of every chunk (one thread per chunk, 64 chains in
// flight per wave); the first kcap records go to the chunk's slots so that an
// accepted chunk is emitted by a parallel copy instead of a second walk
__global__ __launch_bounds__(WALK_T) void walk_spec_kernel(FileTab t, const uint64_t *__restrict__ s_start,
                                                           uint64_t *__restrict__ s_exit, uint32_t *__restrict__ s_count,
                                                           int32_t *__restrict__ s_status, RecSlot *__restrict__ slots,
                                                           uint32_t kcap) {
    const uint64_t w = (uint64_t)blockIdx.x * WALK_T + threadIdx.x;
    if (w >= (uint64_t)t.nfiles * t.cpf)
        return;
    const uint64_t start = s_start[w];
    if (start == NONE)
        return;
    const uint32_t fi = (uint32_t)(w / t.cpf), c = (uint32_t)(w % t.cpf);
    const uint64_t len = t.file_len[fi];
    const uint64_t cend = ((uint64_t)c + 1) << t.lg;
    uint32_t count;
    uint64_t exit;
    int32_t st;
    walk_chain<SPEC>(t.image + t.file_off[fi], len, start, cend, count, exit, st, slots + w * kcap, kcap, 0, 0, 0,
                     nullptr, nullptr, nullptr, nullptr);
    s_exit[w] = exit;
    s_count[w] = count;
    s_status[w] = st;
}

enum ChunkMode : uint32_t { MODE_NONE = 0, MODE_COPY = 1, MODE_WALK = 2 };

// B: exact stitch (one thread per file); re-walks a chunk serially when its
// speculative start is not the true exit of the chunk before it
__global__ __launch_bounds__(WALK_T) void walk_stitch_kernel(FileTab t, const uint64_t *__restrict__ s_start,
                                                             const uint64_t *__restrict__ s_exit,
                                                             const uint32_t *__restrict__ s_count,
                                                             const int32_t *__restrict__ s_status,
                                                             uint64_t *__restrict__ true_start,
                                                             uint64_t *__restrict__ chunk_base,
                                                             uint32_t *__restrict__ chunk_mode, uint32_t kcap,
                                                             uint64_t *__restrict__ file_records,
                                                             int32_t *__restrict__ file_status,
                                                             uint32_t *__restrict__ rewalks) {
    const uint32_t fi = blockIdx.x * WALK_T + threadIdx.x;
    if (fi >= t.nfiles)
        return;
    const uint64_t len = t.file_len[fi];
    const uint8_t *f = t.image + t.file_off[fi];
    const uint64_t w0 = (uint64_t)fi * t.cpf;
    uint64_t total = 0;
    int32_t st = ST_CONTINUE;
    uint64_t pos = 0;
    uint32_t redo = 0;
    if (len > ((uint64_t)t.cpf << t.lg)) { // longer than the caller's max_file_len bound
        st = ZDB_WALK_EXCEEDS_BOUND;
    } else if (s_status[w0] == ZDB_WALK_BAD_DESCRIPTOR) {
        st = ZDB_WALK_BAD_DESCRIPTOR;
    } else {
        pos = ZDB_DATA_HEADER_SIZE; // chunk 0 starts where the reference starts
    }
    for (uint32_t c = 0; c < t.cpf; c++) {
        const uint64_t w = w0 + c;
        const uint64_t cend = ((uint64_t)c + 1) << t.lg;
        chunk_base[w] = total;
        if (st != ST_CONTINUE || pos >= cend) { // walk over, or no record starts in this chunk
            true_start[w] = NONE;
            chunk_mode[w] = MODE_NONE;
            continue;
        }
        true_start[w] = pos;
        uint32_t count;
        uint64_t exit;
        int32_t cs;
        if (s_start[w] == pos) {
            count = s_count[w];
            exit = s_exit[w];
            cs = s_status[w];
            chunk_mode[w] = count <= kcap ? MODE_COPY : MODE_WALK;
        } else {
            walk_chain<COUNT>(f, len, pos, cend, count, exit, cs, nullptr, 0, 0, 0, 0, nullptr, nullptr, nullptr,
                              nullptr);
            chunk_mode[w] = MODE_WALK;
            redo++;
        }
        total += count;
        pos = exit;
        st = cs;
    }
    file_records[fi] = total;
    file_status[fi] = st == ST_CONTINUE ? ZDB_WALK_OK : st;
    rewalks[fi] = redo;
}

// B2: record counts -> global record base of every file, in place
// (exclusive prefix; entry nfiles = total)
__global__ void walk_prefix_kernel(uint32_t nfiles, uint64_t *__restrict__ file_records,
                                   uint32_t *__restrict__ rewalks) {
    if (threadIdx.x != 0 || blockIdx.x != 0)
        return;
    uint64_t acc = 0;
    uint32_t redo = 0;
    for (uint32_t i = 0; i < nfiles; i++) {
        const uint64_t n = file_records[i];
        file_records[i] = acc;
        acc += n;
        redo += rewalks[i];
    }
    file_records[nfiles] = acc;
    rewalks[nfiles] = redo;
}

// C1: descriptors of the accepted chunks, copied from their slots (one
// thread per slot)
__global__ __launch_bounds__(WALK_T) void walk_copy_kernel(FileTab t, const uint32_t *__restrict__ chunk_mode,
                                                           const uint32_t *__restrict__ s_count,
                                                           const RecSlot *__restrict__ slots, uint32_t kcap,
                                                           const uint64_t *__restrict__ chunk_base,
                                                           const uint64_t *__restrict__ file_base, uint64_t capacity,
                                                           uint64_t *__restrict__ entry_off, uint64_t *__restrict__ poff,
                                                           uint32_t *__restrict__ plen,
                                                           uint32_t *__restrict__ expect) {
    const uint64_t g = (uint64_t)blockIdx.x * WALK_T + threadIdx.x;
    const uint64_t w = g / kcap;
    const uint32_t i = (uint32_t)(g % kcap);
    if (w >= (uint64_t)t.nfiles * t.cpf || chunk_mode[w] != MODE_COPY || i >= s_count[w])
        return;
    const uint32_t fi = (uint32_t)(w / t.cpf);
    const uint64_t idx = file_base[fi] + chunk_base[w] + i;
    if (idx >= capacity)
        return;
    const RecSlot r = slots[w * kcap + i];
    const uint64_t foff = t.file_off[fi];
    entry_off[idx] = foff + r.pos;
    poff[idx] = foff + r.pos + r.hlen;
    plen[idx] = r.len;
    expect[idx] = r.expect;
}

// C2: descriptors of the chunks that had to be re-walked, or had more
// records than slots (one thread per chunk)
__global__ __launch_bounds__(WALK_T) void walk_emit_kernel(FileTab t, const uint64_t *__restrict__ true_start,
                                                           const uint32_t *__restrict__ chunk_mode,
                                                           const uint64_t *__restrict__ chunk_base,
                                                           const uint64_t *__restrict__ file_base, uint64_t capacity,
                                                           uint64_t *__restrict__ entry_off, uint64_t *__restrict__ poff,
                                                           uint32_t *__restrict__ plen,
                                                           uint32_t *__restrict__ expect) {
    const uint64_t w = (uint64_t)blockIdx.x * WALK_T + threadIdx.x;
    if (w >= (uint64_t)t.nfiles * t.cpf || chunk_mode[w] != MODE_WALK)
        return;
    const uint32_t fi = (uint32_t)(w / t.cpf), c = (uint32_t)(w % t.cpf);
    const uint64_t cend = ((uint64_t)c + 1) << t.lg;
    const uint64_t foff = t.file_off[fi];
    uint32_t count;
    uint64_t exit;
    int32_t st;
    walk_chain<EMIT>(t.image + foff, t.file_len[fi], true_start[w], cend, count, exit, st, nullptr, 0, foff,
                     file_base[fi] + chunk_base[w], capacity, entry_off, poff, plen, expect);
}

// per (device, stream) workspace of the walk
struct WalkWs {
    void *ptr = nullptr;
    size_t bytes = 0;
};
std::mutex g_walk_mu[64];
std::map<void *, WalkWs> g_walk_ws[64];

} // namespace

extern "C" {

int zdb_datafile_walk_device(const uint8_t *d_image, const uint64_t *d_file_off, const uint64_t *d_file_len,
                             uint32_t nfiles, uint64_t max_file_len, uint32_t chunk_bytes, uint64_t *d_entry_off,
                             uint64_t *d_payload_off, uint32_t *d_payload_len, uint32_t *d_expected,
                             uint64_t capacity, uint64_t *d_file_records, int32_t *d_file_status,
                             uint32_t *d_rewalks, void *stream) {
    if (nfiles == 0)
        return ZDB_CRC32_OK;
    if (!d_image || !d_file_off || !d_file_len || !d_file_records || !d_file_status || !d_rewalks)
        return ZDB_CRC32_EINVAL;
    if (capacity && (!d_entry_off || !d_payload_off || !d_payload_len || !d_expected))
        return ZDB_CRC32_EINVAL;
    uint32_t lg = DEFAULT_LG_CHUNK;
    if (chunk_bytes) {
        if (chunk_bytes < 1024 || (chunk_bytes & (chunk_bytes - 1)))
            return ZDB_CRC32_EINVAL; // a power of two >= 1 KiB (the search step)
        lg = (uint32_t)__builtin_ctz(chunk_bytes);
    }
    if (max_file_len > (1ull << 32)) // datafile offsets are u32 (data.h:59, index.h:54)
        return ZDB_CRC32_EINVAL;
    const uint64_t cpf64 = max_file_len ? (max_file_len + (1ull << lg) - 1) >> lg : 1;
    const uint64_t nchunks = cpf64 * nfiles;
    if (nchunks > (1ull << 31))
        return ZDB_CRC32_EINVAL;
    zdbcrc_internal_mark_hip();
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64)
        return ZDB_CRC32_ENODEV;
    hipStream_t st = static_cast<hipStream_t>(stream);
    std::lock_guard<std::mutex> g(g_walk_mu[dev]);
    // workspace: per chunk s_start, s_exit, true_start, chunk_base (u64),
    // s_count, s_status, chunk_mode (4 B), kcap record slots (16 B each)
    const uint32_t kcap = nchunks <= 65536 ? 512u : 64u;
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    const size_t need = 4 * al(nchunks * 8) + 3 * al(nchunks * 4) + al(nchunks * kcap * sizeof(RecSlot));
    WalkWs &ws = g_walk_ws[dev][stream];
    if (ws.bytes < need) {
        if (ws.ptr) {
            hipStreamSynchronize(st);
            hipFree(ws.ptr);
            ws.ptr = nullptr;
            ws.bytes = 0;
        }
        if (hipMalloc(&ws.ptr, need) != hipSuccess)
            return ZDB_CRC32_ENOMEM;
        ws.bytes = need;
    }
    uint8_t *b = static_cast<uint8_t *>(ws.ptr);
    uint64_t *s_start = reinterpret_cast<uint64_t *>(b);
    uint64_t *s_exit = reinterpret_cast<uint64_t *>(b + al(nchunks * 8));
    uint64_t *true_start = reinterpret_cast<uint64_t *>(b + 2 * al(nchunks * 8));
    uint64_t *chunk_base = reinterpret_cast<uint64_t *>(b + 3 * al(nchunks * 8));
    uint32_t *s_count = reinterpret_cast<uint32_t *>(b + 4 * al(nchunks * 8));
    int32_t *s_status = reinterpret_cast<int32_t *>(b + 4 * al(nchunks * 8) + al(nchunks * 4));
    uint32_t *chunk_mode = reinterpret_cast<uint32_t *>(b + 4 * al(nchunks * 8) + 2 * al(nchunks * 4));
    RecSlot *slots = reinterpret_cast<RecSlot *>(b + 4 * al(nchunks * 8) + 3 * al(nchunks * 4));

    const FileTab t{d_image, d_file_off, d_file_len, nfiles, (uint32_t)cpf64, lg};
    hipLaunchKernelGGL(walk_search_kernel, dim3((uint32_t)nchunks), dim3(WALK_T), 0, st, t, s_start, s_status);
    const dim3 gch((uint32_t)((nchunks + WALK_T - 1) / WALK_T));
    hipLaunchKernelGGL(walk_spec_kernel, gch, dim3(WALK_T), 0, st, t, s_start, s_exit, s_count, s_status, slots,
                       kcap);
    hipLaunchKernelGGL(walk_stitch_kernel, dim3((nfiles + WALK_T - 1) / WALK_T), dim3(WALK_T), 0, st, t, s_start,
                       s_exit, s_count, s_status, true_start, chunk_base, chunk_mode, kcap, d_file_records,
                       d_file_status, d_rewalks);
    hipLaunchKernelGGL(walk_prefix_kernel, dim3(1), dim3(64), 0, st, nfiles, d_file_records, d_rewalks);
    if (capacity) {
        const uint64_t nslots = nchunks * kcap;
        hipLaunchKernelGGL(walk_copy_kernel, dim3((uint32_t)((nslots + WALK_T - 1) / WALK_T)), dim3(WALK_T), 0, st,
                           t, chunk_mode, s_count, slots, kcap, chunk_base, d_file_records, capacity, d_entry_off,
                           d_payload_off, d_payload_len, d_expected);
        hipLaunchKernelGGL(walk_emit_kernel, gch, dim3(WALK_T), 0, st, t, true_start, chunk_mode, chunk_base,
                           d_file_records, capacity, d_entry_off, d_payload_off, d_payload_len, d_expected);
    }
    return hipGetLastError() == hipSuccess ? ZDB_CRC32_OK : ZDB_CRC32_ELAUNCH;
}

int zdb_datafile_scan_device(const uint8_t *d_image, const uint64_t *d_file_off, const uint64_t *d_file_len,
                             uint32_t nfiles, uint64_t max_file_len, uint32_t chunk_bytes,
                             const zdb_scan_buffers_t *b, uint64_t *n_records, void *stream) {
    if (!b || !n_records || !b->file_records || !b->mismatch_count || (b->max_mismatch && !b->mismatch))
        return ZDB_CRC32_EINVAL;
    *n_records = 0;
    int rc = zdb_datafile_walk_device(d_image, d_file_off, d_file_len, nfiles, max_file_len, chunk_bytes,
                                      b->entry_off, b->payload_off, b->payload_len, b->expected, b->capacity,
                                      b->file_records, b->file_status, b->rewalks, stream);
    if (rc)
        return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    uint64_t n = 0;
    if (nfiles) {
        if (hipMemcpyAsync(&n, b->file_records + nfiles, sizeof(n), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return ZDB_CRC32_ELAUNCH;
    }
    *n_records = n;
    if (n > b->capacity)
        return ZDB_CRC32_ENOSPC;
    return zdb_crc32_verify_device(d_image, b->payload_off, b->payload_len, b->expected, b->computed,
                                   b->mismatch, b->mismatch_count, b->max_mismatch, n, stream);
}

} // extern "C"
