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
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

#include <hip/hip_runtime.h>

#include "zdb_crc32.h"
#include "zdb_datafile.h"

extern "C" void zdbcrc_internal_mark_hip(void); // crc32_hip.hip (not exported)
extern "C" int zdbcrc_internal_verify_device_dn(const uint8_t *, const uint64_t *, const uint32_t *, const uint32_t *,
                                                uint32_t *, uint32_t *, uint32_t *, uint32_t, size_t,
                                                const uint64_t *, void *); // crc32_hip.hip (not exported)

namespace {

constexpr uint64_t NONE = ~0ull;
constexpr int32_t ST_CONTINUE = -1;
// 8 MiB chunks: C4 (64 x 256 MiB files of C3 payloads) walks in 0.83 ms
// against 0.91 (4 MiB), 1.28 (2 MiB) and 1.24 ms (16 MiB) --
// profiles/r2/walk_probe.jsonl; smaller chunks search more, larger ones
// follow longer chains
constexpr uint32_t DEFAULT_LG_CHUNK = 23;
constexpr uint32_t WALK_T = 256;
// search: threads per chunk, KiB per wave block; each lane loads its own 16
// bytes only and takes the next 16 from its neighbour (walk 0.58 -> 0.51 ms
// on C4, profiles/r2/walk_search_ab*.jsonl)
// at most 80 VGPRs (6 waves per SIMD instead of 5 at the compiler's 82:
// walk 0.502 -> 0.480 ms with the windowed chain below, profiles/r2/
// walk_occupancy_window_chain_ab.jsonl; 64 VGPRs spill, 4 KiB blocks are slower)
constexpr int SEARCH_T = 256, SEARCH_SU = 8, SEARCH_MW = 6;
// chains per wave (A2, C2): the lanes of a wave hop in lockstep, each hop
// waiting for the slowest of its lanes' header loads, so fewer chains per
// wave on more CUs shorten every hop
constexpr uint32_t CHAINS_PER_WAVE = 16;
// A2 shape: one wave per chunk reading 1 KiB windows (walk_spec_win_kernel)
// instead of one lane per chunk reading each header (C4: walk -1.5 to -3 %
// in two A/B rounds, the same records and exits: GPU walk tests)
constexpr bool WINDOW_CHAIN = true;
// A1 + A2 fused (walk_search_chain_kernel): a chunk's chain starts as soon as
// its own search is done, overlapping the other chunks' searches (C4 walk
// 0.482 -> 0.421 ms in two A/B rounds, profiles/r2/walk_fused_ab.jsonl)
constexpr bool FUSED_WALK = true;
// chain window: 0 = the 1 KiB register window (chain_window), else the bytes
// of the LDS-staged window (chain_wide).  C4 walk 0.432 (register) / 0.409
// (1 KiB) / 0.407 (2 KiB) / 0.425 (4 KiB) / 0.446 ms (8 KiB),
// profiles/r3/walk_chain_window_ab.jsonl
constexpr uint32_t CHAIN_WB = 2048;
// search filter in two passes (scan_block_ilp): no gain (C4 walk 0.423 ->
// 0.434 ms, profiles/r3/walk_search_ilp_ab.jsonl)
constexpr bool SEARCH_ILP = false;
// skewed chunk edges (chunk_edge): C4 walk 0.414 -> 0.402 ms in three A/B
// rounds (profiles/r3/walk_chunk_skew_ab.jsonl)
constexpr bool CHUNK_SKEW = true;

// little-endian u32 at any byte address: two aligned dword loads + one
// v_alignbyte (reads up to 7 bytes past p; images are readable 16 bytes past
// their end, as for the checksum kernel)
typedef const __attribute__((address_space(1))) uint32_t gu32; // global loads, not flat (vmcnt only)

__device__ __forceinline__ uint32_t ld_le32(const uint8_t *p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    gu32 *q = reinterpret_cast<gu32 *>(a & ~uintptr_t(3));
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
        gu32 *q = reinterpret_cast<gu32 *>(a & ~uintptr_t(3));
        const uint32_t sh = (uint32_t)(a & 3);
        const uint32_t q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3], q4 = q[4];
        const uint32_t w0 = __builtin_amdgcn_alignbyte(q1, q0, sh), w1 = __builtin_amdgcn_alignbyte(q2, q1, sh);
        const uint32_t w2 = __builtin_amdgcn_alignbyte(q3, q2, sh), w3 = __builtin_amdgcn_alignbyte(q4, q3, sh);
        return Hdr{w0 & 0xFFu, (w0 >> 8) | (w1 << 24), (w2 >> 8) | (w3 << 24)};
    }
    return Hdr{f[pos], 0u, 0u}; // no whole header fits: the walk stops on SHORT_HEADER
}

// the same in two halves, so that a chain can issue the next header's loads
// and decode them only after this record's stores have been issued
// (branch-free: a load under a branch makes the compiler wait for it where
// the branches join).  Within 4 bytes of the file's end no whole header
// fits: the window then starts 4 bytes earlier, so that it stays within the
// 16 readable bytes past the end, and only idlength is decoded (the walk
// stops on SHORT_HEADER); pos >= 28 always (the walk starts at or after the
// 28-byte datafile header)
struct RawHdr {
    uint32_t q0, q1, q2, q3, q4, sh; // sh > 3: window shifted back 4 bytes
};
__device__ __forceinline__ RawHdr load_raw(const uint8_t *f, uint64_t len, uint64_t pos) {
    const uint32_t back = pos + 4 <= len ? 0u : 4u;
    const uintptr_t a = reinterpret_cast<uintptr_t>(f + pos);
    gu32 *q = reinterpret_cast<gu32 *>((a & ~uintptr_t(3)) - back);
    return RawHdr{q[0], q[1], q[2], q[3], q[4], (uint32_t)(a & 3) + back};
}
__device__ __forceinline__ Hdr decode(const RawHdr &r) {
    if (r.sh > 3)
        return Hdr{__builtin_amdgcn_alignbyte(r.q2, r.q1, r.sh - 4) & 0xFFu, 0u, 0u};
    const uint32_t w0 = __builtin_amdgcn_alignbyte(r.q1, r.q0, r.sh), w1 = __builtin_amdgcn_alignbyte(r.q2, r.q1, r.sh);
    const uint32_t w2 = __builtin_amdgcn_alignbyte(r.q3, r.q2, r.sh), w3 = __builtin_amdgcn_alignbyte(r.q4, r.q3, r.sh);
    return Hdr{w0 & 0xFFu, (w0 >> 8) | (w1 << 24), (w2 >> 8) | (w3 << 24)};
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
// The next header's loads are issued before this record's stores: the
// memory counter completes in order, so a store issued first would add its
// own round trip to every hop of the chain (2.4 -> ~1.2 us per hop).
template <int MODE>
__device__ __forceinline__ void walk_chain(const uint8_t *f, uint64_t len, uint64_t pos, uint64_t cend,
                                           uint32_t &count, uint64_t &exit, int32_t &st, RecSlot *slots,
                                           uint32_t kcap, uint64_t foff, uint64_t idx, uint64_t capacity,
                                           uint64_t *__restrict__ entry_off, uint64_t *__restrict__ poff,
                                           uint32_t *__restrict__ plen, uint32_t *__restrict__ expect) {
    count = 0;
    st = ST_CONTINUE;
    RawHdr raw{0u, 0u, 0u, 0u, 0u, 4u};
    if (pos < cend && pos < len)
        raw = load_raw(f, len, pos);
    while (pos < cend) {
        if (pos >= len) { // clean end of file (pos == len)
            st = ZDB_WALK_OK;
            break;
        }
        // the header at pos (hop of datafile.c zdb_datafile_walk)
        const Hdr h = decode(raw);
        const uint32_t hlen = ZDB_ENTRY_HEADER_SIZE + h.idl;
        if (pos + hlen > len) {
            st = ZDB_WALK_SHORT_HEADER;
            break;
        }
        const uint32_t L = h.L;
        uint64_t next = pos + hlen;
        int32_t s = ST_CONTINUE;
        if (L) {
            if (next + L > len)
                s = ZDB_WALK_SHORT_PAYLOAD;
            else
                next += L;
        }
        // the next header (decoded at the top of the next hop, after the stores
        // below); unconditional -- at the end of the walk it reloads pos
        raw = load_raw(f, len, s == ST_CONTINUE && next < len ? next : pos);
        __asm__ volatile("" ::: "memory"); // keep the loads above ahead of the stores below
        if (MODE != COUNT) {
            const bool full = s == ST_CONTINUE && L > 0; // payload present and non-empty
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

// relaxed confirmation (files whose `previous` fields do not chain, e.g. not
// written by zdbd): the header at p and the RELAXED_HOPS headers its chain
// leads to all pass the byte filter (datalength < 2^24, flags <= 3) and fit
// in the file, or the chain ends exactly at the end of the file.  A random
// position passes one hop with p ~ 2^-14, so three hops make a false start
// practically impossible on non-adversarial data -- and a false start only
// costs a serial re-walk: the stitch still checks every chunk start.
constexpr int RELAXED_HOPS = 3;
__device__ __forceinline__ bool forward_ok(const uint8_t *f, uint64_t len, uint64_t p) {
    for (int hop = 0; hop <= RELAXED_HOPS; hop++) {
        if (p == len)
            return true;
        if (p + ZDB_ENTRY_HEADER_SIZE > len)
            return false;
        const uintptr_t a = reinterpret_cast<uintptr_t>(f + p);
        gu32 *q = reinterpret_cast<gu32 *>(a & ~uintptr_t(3));
        const uint32_t sh = (uint32_t)(a & 3);
        const uint32_t q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3], q4 = q[4];
        const uint32_t w0 = __builtin_amdgcn_alignbyte(q1, q0, sh), w1 = __builtin_amdgcn_alignbyte(q2, q1, sh);
        const uint32_t w3 = __builtin_amdgcn_alignbyte(q4, q3, sh);
        const uint32_t idl = w0 & 0xFFu, L = (w0 >> 8) | (w1 << 24), flags = (w3 >> 8) & 0xFFu;
        if ((L >> 24) != 0 || flags > 3u)
            return false;
        const uint64_t next = p + ZDB_ENTRY_HEADER_SIZE + idl + L;
        if (next > len)
            return false;
        p = next;
    }
    return true;
}

struct FileTab {
    const uint8_t *image;
    const uint64_t *file_off;
    const uint64_t *file_len;
    uint32_t nfiles;
    uint32_t cpf;  // chunks per file (grid)
    uint32_t lg;   // log2 chunk bytes
    uint32_t skew; // chunk edges moved down by up to 1/8 chunk (see chunk_edge)
};

// file-relative start of chunk c of file fi (c == cpf: the end of the last
// chunk).  With t.skew, every inner edge moves down by a pseudo-random
// multiple of 4 KiB below 1/8 chunk: the concurrent searches, which all start
// at their chunk edge and step outward by the same block sizes, then spread
// over the memory channels instead of hitting addresses equal modulo the
// chunk size (edges stay increasing; any edges give the same walk -- the
// stitch joins chunks whatever their bounds)
__device__ __forceinline__ uint64_t chunk_edge(const FileTab &t, uint32_t fi, uint64_t c) {
    const uint64_t e = c << t.lg;
    if (!t.skew || c == 0 || c >= t.cpf || t.lg < 16)
        return e;
    const uint32_t h = (uint32_t)(((uint64_t)fi * t.cpf + c) * 0x9E3779B1u) >> 8;
    return e - (uint64_t)(h % (1u << (t.lg - 15))) * 4096u;
}

// candidate positions among the 16 starting at a 16-byte block whose 32
// bytes are d[0..7]: byte p+4 (top byte of datalength) is 0 and byte p+13
// (flags) is <= 3.  One zero-byte test covers 4 positions: bit 8r+7 of z[j]
// is set when position 4j+r qualifies (the test has no false negatives;
// false positives only cost a back-pointer check).
__device__ __forceinline__ uint32_t haszero(uint32_t x) { return (x - 0x01010101u) & ~x & 0x80808080u; }

// OR1: both byte tests in one zero-byte test -- byte r of (datalength top
// byte | flags & 0xFC) is zero iff both are (5 VALU per 4 positions instead
// of 9; haszero's false positives differ, its hits on zero bytes do not)
constexpr bool FILTER_OR = true;
template <bool OR1 = FILTER_OR>
__device__ __forceinline__ void candidates(const uint32_t (&d)[8], uint32_t (&z)[4]) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t fl = __builtin_amdgcn_alignbyte(d[j + 4], d[j + 3], 1u); // bytes 4j+13 .. 4j+16
        z[j] = OR1 ? haszero(d[j + 1] | (fl & 0xFCFCFCFCu)) : haszero(d[j + 1]) & haszero(fl & 0xFCFCFCFCu);
    }
}

// verified candidates of the SB-byte block at b (16-byte aligned) among the
// positions [lo, hi): FWD -> the lowest (NONE if none), else the highest (0
// if none).  Wave-uniform result.  Loads read [p0, p0 + 32) for every lane
// whose 16 positions meet [lo, hi) (p0 >= 16 whenever lo >= 28, and at most 32
// bytes past hi: within the file, or within the 16 readable bytes past it)
// NOA1: each lane loads its own 16 bytes only and takes the following 16
// from the next lane (DPP wave shift; lane 63 from lane 0 of the next 1 KiB,
// or from one extra load after the block)
__device__ __forceinline__ uint32_t from_next_lane(uint32_t own_next_row0, uint32_t v, uint32_t lane) {
    const uint32_t sh = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, false); // wave_shl:1
    return lane == 63 ? own_next_row0 : sh;
}

// RELAXED: candidates confirmed by forward_ok instead of the back-pointer
// (and without the `previous` < p test)
template <bool FWD, int SU, bool NOA1 = false, bool RELAXED = false, bool OR1 = FILTER_OR>
__device__ __forceinline__ uint64_t scan_block(const uint8_t *f, uint64_t len, uint64_t b, uint64_t lo, uint64_t hi,
                                               uint32_t lane) {
    uint4 a0[SU], a1[NOA1 ? 1 : SU], tl = make_uint4(~0u, ~0u, ~0u, ~0u);
#pragma unroll
    for (int u = 0; u < SU; u++) { // every load of the block in flight
        const uint64_t p0 = b + 1024u * u + 16u * lane;
        if (NOA1) { // also the 16 bytes the previous lane's positions need
            a0[u] = p0 + 32 > lo && p0 < hi + 16 ? *reinterpret_cast<const uint4 *>(f + p0)
                                                  : make_uint4(~0u, ~0u, ~0u, ~0u);
        } else if (p0 + 16 > lo && p0 < hi) {
            a0[u] = *reinterpret_cast<const uint4 *>(f + p0);
            a1[u] = *reinterpret_cast<const uint4 *>(f + p0 + 16);
        } else {
            a0[u] = a1[u] = make_uint4(~0u, ~0u, ~0u, ~0u); // no candidate
        }
    }
    // the 16 bytes after the block, for lane 63 of the last row.  The address
    // is wave-uniform and not 4-byte aligned in general (files sit at any
    // offset of the image): it must stay a vector load -- as a scalar load
    // (which the compiler chose in the 128-thread shape) the low address
    // bits are dropped and the bytes are wrong (walk_search_ab3-5)
    if (NOA1 && b + 1024u * SU < hi + 16) {
        uint64_t ta = reinterpret_cast<uint64_t>(f + b + 1024u * SU);
        __asm__ volatile("" : "+v"(ta)); // keep the address in a VGPR
        tl = *reinterpret_cast<const uint4 *>(ta);
    }
    uint64_t found = FWD ? NONE : 0;
#pragma unroll
    for (int u = 0; u < SU; u++) {
        const uint64_t p0 = b + 1024u * u + 16u * lane;
        uint4 nx;
        if (NOA1) {
            const uint4 r0 = u + 1 < SU ? make_uint4(__builtin_amdgcn_readlane(a0[u + 1 < SU ? u + 1 : u].x, 0),
                                                     __builtin_amdgcn_readlane(a0[u + 1 < SU ? u + 1 : u].y, 0),
                                                     __builtin_amdgcn_readlane(a0[u + 1 < SU ? u + 1 : u].z, 0),
                                                     __builtin_amdgcn_readlane(a0[u + 1 < SU ? u + 1 : u].w, 0))
                                        : tl;
            nx = make_uint4(from_next_lane(r0.x, a0[u].x, lane), from_next_lane(r0.y, a0[u].y, lane),
                            from_next_lane(r0.z, a0[u].z, lane), from_next_lane(r0.w, a0[u].w, lane));
        } else {
            nx = a1[NOA1 ? 0 : u];
        }
        const uint32_t d[8] = {a0[u].x, a0[u].y, a0[u].z, a0[u].w, nx.x, nx.y, nx.z, nx.w};
        uint32_t z[4];
        candidates<OR1>(d, z);
        if (z[0] | z[1] | z[2] | z[3]) { // rare: confirm through the successor's back-pointer
#pragma unroll
            for (int j = 0; j < 4; j++) {
                uint32_t m = z[j];
                while (m && (!FWD || found == NONE)) {
                    const uint32_t r = (uint32_t)__builtin_ctz(m) >> 3;
                    m &= ~(0xFFu << (8 * r));
                    const uint64_t p = p0 + 4u * j + r;
                    // the entry's own `previous` (bytes p+5..p+8, still in
                    // registers) must lie before it: every entry but a file's
                    // first (offset 28, never a candidate here) points back at
                    // the entry written just before it (data.c:601).  ~2^-5 of
                    // the filter's false hits pass, so the header loads below
                    // stay rare
                    const uint32_t prev = r == 3 ? d[j + 2] : __builtin_amdgcn_alignbyte(d[j + 2], d[j + 1], r + 1);
                    if (RELAXED) {
                        if (p >= lo && p < hi && forward_ok(f, len, p))
                            found = p;
                    } else if (p >= lo && p < hi && (uint64_t)prev < p) {
                        const Hdr h = load_hdr(f, len, p);
                        if (plausible_successor(f, len, p, h.idl, h.L))
                            found = p; // positions rise within a lane: the last is the highest
                    }
                }
            }
        }
        if (FWD) {
            const uint64_t hit = __ballot(found != NONE);
            if (hit) { // lanes hold increasing addresses: the lowest lane has the block's first candidate
                const uint32_t l = (uint32_t)__builtin_ctzll(hit);
                return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(found >> 32), l) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane((uint32_t)found, l); // int results: no sign extension
            }
        }
    }
    if (FWD)
        return NONE;
    // highest over the wave (positions < 4 GiB: datafile offsets are u32)
    uint32_t x = (uint32_t)found;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t y = (uint32_t)__shfl_xor((int)x, o, 64);
        x = y > x ? y : x;
    }
    return x;
}

// one 1 KiB row of a scan block: this lane's 16 bytes, the next lane's 16
// (lane 63: lane 0 of the next row, `next`, uniform after readlane) and the
// filter of its 16 positions
__device__ __forceinline__ void filter_row(const uint4 &cur, const uint4 &next, uint32_t lane, uint32_t (&d)[8],
                                           uint32_t (&z)[4]) {
    d[0] = cur.x;
    d[1] = cur.y;
    d[2] = cur.z;
    d[3] = cur.w;
    d[4] = from_next_lane(__builtin_amdgcn_readlane(next.x, 0), cur.x, lane);
    d[5] = from_next_lane(__builtin_amdgcn_readlane(next.y, 0), cur.y, lane);
    d[6] = from_next_lane(__builtin_amdgcn_readlane(next.z, 0), cur.z, lane);
    d[7] = from_next_lane(__builtin_amdgcn_readlane(next.w, 0), cur.w, lane);
    candidates(d, z);
}

// scan_block (NOA1 shape) in two passes: the byte filter over all SU rows
// first, with no branch between them (the rows' dependency chains -- DPP
// neighbour, readlane, filter -- interleave instead of ending each in a
// ballot and a branch), then, only when some lane of the block has a
// candidate, the confirmation row by row in address order as scan_block does.
// Same result as scan_block<FWD, SU, true, RELAXED>.
template <bool FWD, int SU, bool RELAXED = false, bool ILP_PAIR = true>
__device__ __forceinline__ uint64_t scan_block_ilp(const uint8_t *f, uint64_t len, uint64_t b, uint64_t lo,
                                                   uint64_t hi, uint32_t lane) {
    uint4 a0[SU], tl = make_uint4(~0u, ~0u, ~0u, ~0u);
#pragma unroll
    for (int u = 0; u < SU; u++) {
        const uint64_t p0 = b + 1024u * u + 16u * lane;
        a0[u] = p0 + 32 > lo && p0 < hi + 16 ? *reinterpret_cast<const uint4 *>(f + p0)
                                              : make_uint4(~0u, ~0u, ~0u, ~0u);
    }
    if (b + 1024u * SU < hi + 16) { // see scan_block: must stay a vector load
        uint64_t ta = reinterpret_cast<uint64_t>(f + b + 1024u * SU);
        __asm__ volatile("" : "+v"(ta));
        tl = *reinterpret_cast<const uint4 *>(ta);
    }
    uint32_t any = 0;
#pragma unroll
    for (int u = 0; u < SU; u++) {
        uint32_t d[8], z[4];
        filter_row(a0[u], u + 1 < SU ? a0[u + 1 < SU ? u + 1 : u] : tl, lane, d, z);
        any |= ((z[0] | z[1] | z[2] | z[3]) != 0u ? 1u : 0u) << u;
        if (ILP_PAIR && (u & 1)) // at most two rows in flight (80 VGPRs)
            __builtin_amdgcn_sched_barrier(0);
    }
    uint64_t found = FWD ? NONE : 0;
    if (__ballot(any != 0u)) {
#pragma unroll
        for (int u = 0; u < SU; u++) {
            if (!__ballot((any >> u) & 1u))
                continue;
            // the row's 32 bytes per lane again (L2-hot; keeping a0 live
            // through this rare pass costs the hot pass its registers), with
            // the first pass's bounds: ~0 where nothing was loaded
            const uint64_t p0 = b + 1024u * u + 16u * lane;
            uint4 x0 = make_uint4(~0u, ~0u, ~0u, ~0u), x1 = x0;
            if (p0 + 32 > lo && p0 < hi + 16)
                x0 = *reinterpret_cast<const uint4 *>(f + p0);
            if (p0 + 48 > lo && p0 < hi)
                x1 = *reinterpret_cast<const uint4 *>(f + p0 + 16);
            uint32_t d[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w}, z[4];
            candidates(d, z);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                uint32_t m = z[j];
                while (m && (!FWD || found == NONE)) {
                    const uint32_t r = (uint32_t)__builtin_ctz(m) >> 3;
                    m &= ~(0xFFu << (8 * r));
                    const uint64_t p = p0 + 4u * j + r;
                    const uint32_t prev =
                        r == 3 ? d[j + 2] : __builtin_amdgcn_alignbyte(d[j + 2], d[j + 1], r + 1);
                    if (RELAXED) {
                        if (p >= lo && p < hi && forward_ok(f, len, p))
                            found = p;
                    } else if (p >= lo && p < hi && (uint64_t)prev < p) {
                        const Hdr h = load_hdr(f, len, p);
                        if (plausible_successor(f, len, p, h.idl, h.L))
                            found = p;
                    }
                }
            }
            if (FWD) {
                const uint64_t hit = __ballot(found != NONE);
                if (hit) {
                    const uint32_t l = (uint32_t)__builtin_ctzll(hit);
                    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(found >> 32), l) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((uint32_t)found, l);
                }
            }
        }
    }
    if (FWD)
        return NONE;
    uint32_t x = (uint32_t)found;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t y = (uint32_t)__shfl_xor((int)x, o, 64);
        x = y > x ? y : x;
    }
    return x;
}

// A1: speculative start of every chunk: the first entry header at or past the
// chunk start c0 (one workgroup of NWS waves per chunk).  Half of the waves
// search forward from c0 in interleaved SU-KiB blocks; the other half search
// backward from c0 for the header of the entry that straddles it, whose end
// is the answer.  A chunk start falls inside a payload far more often than
// not (most bytes are in the large values), uniformly within it, so the
// nearer of the two ends is found in half the scanning on average and in
// the worst case.
// the search of chunk w (one workgroup of NT threads); every thread returns
// the chunk's speculative start and status
template <int NT, int SU, bool NOA1, bool ILP = false>
__device__ __forceinline__ void search_chunk(const FileTab &t, uint64_t w, uint64_t &start, int32_t &status) {
    constexpr uint32_t NWS = NT / 64, NF = NWS / 2, NB = NWS - NF;
    constexpr uint64_t SB = 1024u * SU; // bytes per wave block
    __shared__ unsigned long long bestf;
    __shared__ unsigned int bestb;
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    const uint32_t fi = (uint32_t)(w / t.cpf), c = (uint32_t)(w % t.cpf);
    const uint64_t len = t.file_len[fi];
    const uint8_t *f = t.image + t.file_off[fi];
    const uint64_t c0 = chunk_edge(t, fi, c), c1 = chunk_edge(t, fi, (uint64_t)c + 1);
    status = ST_CONTINUE;
    if (c == 0) {
        // data_descriptor_load / _validate (data.c:177-209): 28-byte
        // header, magic "DAT0", version 3
        const bool bad = len < ZDB_DATA_HEADER_SIZE || f[0] != 'D' || f[1] != 'A' || f[2] != 'T' ||
                         f[3] != '0' || ld_le32(f + 4) != ZDB_DATAFILE_VERSION;
        start = bad ? NONE : (uint64_t)ZDB_DATA_HEADER_SIZE;
        status = bad ? ZDB_WALK_BAD_DESCRIPTOR : ST_CONTINUE;
        return;
    }
    start = NONE;
    if (c0 >= len || len < ZDB_ENTRY_HEADER_SIZE)
        return;
    // positions p in [c0, c1) with a whole 18-byte header in the file
    const uint64_t lim = (c1 < len - (ZDB_ENTRY_HEADER_SIZE - 1)) ? c1 : len - (ZDB_ENTRY_HEADER_SIZE - 1);
    constexpr uint64_t LO = ZDB_DATA_HEADER_SIZE; // entries start at or after the datafile header
    if (threadIdx.x == 0) {
        bestf = NONE;
        bestb = 0u;
    }
    __syncthreads();
    bool back = true; // the backward search is still useful (block-uniform)
    for (uint64_t k = 0;; k++) {
        if (wid < NF) {
            const uint64_t b = c0 + (k * NF + wid) * SB;
            if (b < lim) {
                const uint64_t found = ILP ? scan_block_ilp<true, SU>(f, len, b, c0, lim, lane)
                                           : scan_block<true, SU, NOA1>(f, len, b, c0, lim, lane);
                if (found != NONE && lane == 0)
                    atomicMin(&bestf, (unsigned long long)found);
            }
        } else if (back) {
            const uint64_t dist = (k * NB + (wid - NF) + 1) * SB; // block [c0 - dist, c0 - dist + SB)
            if (dist < c0 + SB && c0 + SB - dist > LO) {
                const uint64_t b = c0 > dist ? c0 - dist : 0;
                const uint64_t found = ILP ? scan_block_ilp<false, SU>(f, len, b, LO, c0, lane)
                                           : scan_block<false, SU, NOA1>(f, len, b, LO, c0, lane);
                if (found && lane == 0)
                    atomicMax(&bestb, (unsigned int)found);
            }
        }
        __syncthreads();
        const uint64_t bf = bestf;
        const uint64_t bb = bestb;
        __syncthreads();
        uint64_t ans = NONE;
        bool done = false;
        if (bf != NONE) { // the first header at or past c0
            ans = bf;
            done = true;
        } else if (back && bb) { // the highest header before c0: its entry ends at the answer
            const Hdr h = load_hdr(f, len, bb);
            const uint64_t e = bb + ZDB_ENTRY_HEADER_SIZE + h.idl + h.L;
            if (e >= c0) {
                ans = e < lim ? e : NONE; // no entry starts in this chunk when it ends past it
                done = true;
            } else {
                back = false; // not the straddling entry (a chain the filter cannot see): forward only
            }
        }
        if (!done && c0 + (k + 1) * NF * SB >= lim)
            done = true; // no header in [c0, lim)
        if (back && (k + 1) * NB * SB >= c0 + SB - LO)
            back = false; // reached the datafile header
        if (done) {
            start = ans;
            break;
        }
    }
    if (start != NONE)
        return;
    // No header the back-pointer confirms starts in this chunk: either one
    // entry covers it, or the file's `previous` fields do not chain (a file
    // zdbd did not write) -- every chunk of such a file would otherwise be
    // re-walked serially by the stitch.  Second pass, forward only, with the
    // relaxed confirmation (forward_ok); zdbd's own files never get here
    // unless a single entry spans the whole chunk.
    for (uint64_t k = 0;; k++) {
        const uint64_t b = c0 + (k * NWS + wid) * SB;
        if (b < lim) {
            const uint64_t found = scan_block<true, SU, NOA1, true>(f, len, b, c0, lim, lane); // rare pass
            if (found != NONE && lane == 0)
                atomicMin(&bestf, (unsigned long long)found);
        }
        __syncthreads();
        const uint64_t bf = bestf;
        __syncthreads();
        if (bf != NONE || c0 + (k + 1) * NWS * SB >= lim) {
            start = bf;
            return;
        }
    }
}

template <int NT, int SU, bool NOA1 = false, int MW = 1>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(MW))) void walk_search_kernel(
    FileTab t, uint64_t *__restrict__ s_start, int32_t *__restrict__ s_status) {
    uint64_t start;
    int32_t status;
    search_chunk<NT, SU, NOA1>(t, blockIdx.x, start, status);
    if (threadIdx.x == 0) {
        s_start[blockIdx.x] = start;
        s_status[blockIdx.x] = status;
    }
}

// A2: speculative chain of every chunk (one lane per chunk, CHAINS_PER_WAVE
// chains per one-wave workgroup); the first kcap records go to the chunk's
// slots so that an accepted chunk is emitted by a parallel copy instead of a
// second walk
__global__ __launch_bounds__(64) void walk_spec_kernel(FileTab t, const uint64_t *__restrict__ s_start,
                                                       uint64_t *__restrict__ s_exit, uint32_t *__restrict__ s_count,
                                                       int32_t *__restrict__ s_status, RecSlot *__restrict__ slots,
                                                       uint32_t kcap, uint32_t cpw) {
    const uint64_t w = (uint64_t)blockIdx.x * cpw + threadIdx.x;
    if (threadIdx.x >= cpw || w >= (uint64_t)t.nfiles * t.cpf)
        return;
    const uint64_t start = s_start[w];
    if (start == NONE)
        return;
    const uint32_t fi = (uint32_t)(w / t.cpf), c = (uint32_t)(w % t.cpf);
    const uint64_t len = t.file_len[fi];
    const uint64_t cend = chunk_edge(t, fi, (uint64_t)c + 1);
    uint32_t count;
    uint64_t exit;
    int32_t st;
    walk_chain<SPEC>(t.image + t.file_off[fi], len, start, cend, count, exit, st, slots + w * kcap, kcap, 0, 0, 0,
                     nullptr, nullptr, nullptr, nullptr);
    s_exit[w] = exit;
    s_count[w] = count;
    s_status[w] = st;
}

// A2 with a 1 KiB window per round trip (one wave per chunk): lane l holds
// bytes [16 l, 16 l + 16) of the window that starts at the 16-byte block of
// the current header, so every header that lies inside the window (C3 sizes:
// the records of the small buckets, 64 B - 1 KiB, two thirds of all records)
// is decoded from registers (readlane) instead of a dependent HBM round trip.
// Same records, exits and terminal states as walk_chain<SPEC> -- the bytes
// are the same, only fetched in larger pieces: a header whose 13 decoded
// bytes [pos, pos + 13) reach past the window is fetched by a new window at
// pos; lanes whose 16-byte block starts past the file's end load nothing
// (the image is readable 16 bytes past a file's end, not more), and such
// bytes only matter for a header that cannot fit (SHORT_HEADER either way).
struct Window {
    uint4 v;        // this lane's 16 bytes
    uintptr_t base; // image address of lane 0's block (16-aligned), uniform
};

__device__ __forceinline__ void load_window(Window &w, const uint8_t *f, uint64_t len, uint64_t pos, uint32_t lane) {
    w.base = reinterpret_cast<uintptr_t>(f + pos) & ~uintptr_t(15);
    const uintptr_t a = w.base + 16u * lane;
    const uintptr_t end = reinterpret_cast<uintptr_t>(f + len);
    w.v = make_uint4(0, 0, 0, 0);
    if (a <= end) {
        typedef const __attribute__((address_space(1))) uint32_t gx4 __attribute__((ext_vector_type(4)));
        const auto x = *reinterpret_cast<gx4 *>(a);
        w.v = make_uint4(x.x, x.y, x.z, x.w);
    }
}

// the header fields at window byte offset off (uniform, off + 13 <= 1024)
__device__ __forceinline__ Hdr window_hdr(const Window &w, uint32_t off) {
    const uint32_t a = off >> 4, b = a < 63 ? a + 1 : a;
    uint32_t d[8] = {(uint32_t)__builtin_amdgcn_readlane(w.v.x, a), (uint32_t)__builtin_amdgcn_readlane(w.v.y, a),
                     (uint32_t)__builtin_amdgcn_readlane(w.v.z, a), (uint32_t)__builtin_amdgcn_readlane(w.v.w, a),
                     (uint32_t)__builtin_amdgcn_readlane(w.v.x, b), (uint32_t)__builtin_amdgcn_readlane(w.v.y, b),
                     (uint32_t)__builtin_amdgcn_readlane(w.v.z, b), (uint32_t)__builtin_amdgcn_readlane(w.v.w, b)};
    const uint32_t k = (off & 15u) >> 2, sh = 8u * (off & 3u);
    if (k & 2u) {
#pragma unroll
        for (int i = 0; i < 6; i++)
            d[i] = d[i + 2];
    }
    if (k & 1u) {
#pragma unroll
        for (int i = 0; i < 5; i++)
            d[i] = d[i + 1];
    }
    uint32_t q[4];
#pragma unroll
    for (int i = 0; i < 4; i++)
        q[i] = (uint32_t)((((uint64_t)d[i + 1] << 32) | d[i]) >> sh);
    return Hdr{q[0] & 0xFFu, (q[0] >> 8) | (q[1] << 24), (q[2] >> 8) | (q[3] << 24)};
}

__device__ __forceinline__ bool in_window(const Window &w, const uint8_t *f, uint64_t pos) {
    return reinterpret_cast<uintptr_t>(f + pos) - w.base + 13u <= 1024u;
}

// the windowed chain of chunk w from its speculative start (one wave)
__device__ __forceinline__ uint32_t chain_window(const FileTab &t, uint64_t w, uint64_t start, uint32_t lane,
                                             uint64_t *__restrict__ s_exit, uint32_t *__restrict__ s_count,
                                             int32_t *__restrict__ s_status, RecSlot *__restrict__ slots,
                                             uint32_t kcap) {
    const uint32_t fi = (uint32_t)(w / t.cpf), c = (uint32_t)(w % t.cpf);
    const uint64_t len = t.file_len[fi];
    const uint8_t *f = t.image + t.file_off[fi];
    const uint64_t cend = chunk_edge(t, fi, (uint64_t)c + 1);
    RecSlot *sl = slots + w * kcap;
    uint32_t count = 0;
    int32_t st = ST_CONTINUE;
    uint64_t pos = start;
    Window win;
    uint32_t loads = 0;
    if (pos < cend && pos < len) {
        load_window(win, f, len, pos, lane);
        loads++;
    }
    while (pos < cend) {
        if (pos >= len) { // clean end of file (pos == len)
            st = ZDB_WALK_OK;
            break;
        }
        const Hdr h = window_hdr(win, (uint32_t)(reinterpret_cast<uintptr_t>(f + pos) - win.base));
        const uint32_t hlen = ZDB_ENTRY_HEADER_SIZE + h.idl;
        if (pos + hlen > len) {
            st = ZDB_WALK_SHORT_HEADER;
            break;
        }
        const uint32_t L = h.L;
        uint64_t next = pos + hlen;
        int32_t s = ST_CONTINUE;
        if (L) {
            if (next + L > len)
                s = ZDB_WALK_SHORT_PAYLOAD;
            else
                next += L;
        }
        // the next header's window, when it is not this one (issued before the
        // slot store: the memory counter completes in order)
        if (s == ST_CONTINUE && next < len && next < cend && !in_window(win, f, next)) {
            load_window(win, f, len, next, lane);
            loads++;
        }
        __asm__ volatile("" ::: "memory");
        if (count < kcap && lane == 0) {
            const bool full = s == ST_CONTINUE && L > 0;
            sl[count] = RecSlot{(uint32_t)pos, full ? L : 0u, full ? h.integ : 0u, hlen};
        }
        count++;
        if (s == ZDB_WALK_SHORT_PAYLOAD) {
            st = s;
            break;
        }
        pos = next;
    }
    if (st == ST_CONTINUE && pos >= len)
        st = ZDB_WALK_OK;
    if (lane == 0) {
        s_exit[w] = pos;
        s_count[w] = count;
        s_status[w] = st;
    }
    return loads;
}

// the windowed chain with WB-byte windows staged through LDS (WB / 1024
// 16-byte loads per lane; C4's median entry is ~300 bytes, so a wider window
// decodes more of a chunk's headers without a new round trip: 1 / 2 / 4 /
// 8 KiB windows take 68 / 55 / 45 / 37 window loads per 8 MiB chunk).  Lane l
// loads window bytes [16 (l + 64 j), +16) for j < WB / 1024, each only when
// its block starts at or before the file's end (the 16 readable bytes past
// it), and writes them to the same offset of the wave's LDS window; a header
// is then five uniform LDS dwords.  Same records, exits and terminal states
// as chain_window.
template <uint32_t WB> struct WideWindow {
    static constexpr uint32_t NJ = WB / 1024;
    uint4 v[NJ];
    uintptr_t base;
};

template <uint32_t WB>
__device__ __forceinline__ void load_wide(WideWindow<WB> &w, const uint8_t *f, uint64_t len, uint64_t pos,
                                          uint32_t lane) {
    w.base = reinterpret_cast<uintptr_t>(f + pos) & ~uintptr_t(15);
    const uintptr_t end = reinterpret_cast<uintptr_t>(f + len);
#pragma unroll
    for (uint32_t j = 0; j < WideWindow<WB>::NJ; j++) {
        const uintptr_t a = w.base + 16u * (lane + 64u * j);
        w.v[j] = make_uint4(0, 0, 0, 0);
        if (a <= end) {
            typedef const __attribute__((address_space(1))) uint32_t gx4 __attribute__((ext_vector_type(4)));
            const auto x = *reinterpret_cast<gx4 *>(a);
            w.v[j] = make_uint4(x.x, x.y, x.z, x.w);
        }
    }
}

template <uint32_t WB>
__device__ __forceinline__ void stage_wide(const WideWindow<WB> &w, uint32_t *lds, uint32_t lane) {
#pragma unroll
    for (uint32_t j = 0; j < WideWindow<WB>::NJ; j++)
        *reinterpret_cast<uint4 *>(lds + 4u * (lane + 64u * j)) = w.v[j];
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ Hdr lds_hdr(const uint32_t *lds, uint32_t off) {
    const uint32_t *q = lds + (off >> 2);
    const uint32_t sh = off & 3u;
    const uint32_t q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3], q4 = q[4];
    const uint32_t w0 = __builtin_amdgcn_alignbyte(q1, q0, sh), w1 = __builtin_amdgcn_alignbyte(q2, q1, sh);
    const uint32_t w2 = __builtin_amdgcn_alignbyte(q3, q2, sh), w3 = __builtin_amdgcn_alignbyte(q4, q3, sh);
    return Hdr{w0 & 0xFFu, (w0 >> 8) | (w1 << 24), (w2 >> 8) | (w3 << 24)};
}

template <uint32_t WB>
__device__ __forceinline__ uint32_t chain_wide(const FileTab &t, uint64_t w, uint64_t start, uint32_t lane,
                                           uint64_t *__restrict__ s_exit, uint32_t *__restrict__ s_count,
                                           int32_t *__restrict__ s_status, RecSlot *__restrict__ slots,
                                           uint32_t kcap) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[WB / 4 + 4]; // + the 5th dword of a header at WB - 13
    const uint32_t fi = (uint32_t)(w / t.cpf), c = (uint32_t)(w % t.cpf);
    const uint64_t len = t.file_len[fi];
    const uint8_t *f = t.image + t.file_off[fi];
    const uint64_t cend = chunk_edge(t, fi, (uint64_t)c + 1);
    RecSlot *sl = slots + w * kcap;
    uint32_t count = 0;
    int32_t st = ST_CONTINUE;
    uint64_t pos = start;
    WideWindow<WB> win;
    uint32_t loads = 0;
    if (pos < cend && pos < len) {
        load_wide<WB>(win, f, len, pos, lane);
        stage_wide<WB>(win, lds, lane);
        loads++;
    }
    while (pos < cend) {
        if (pos >= len) { // clean end of file (pos == len)
            st = ZDB_WALK_OK;
            break;
        }
        const Hdr h = lds_hdr(lds, (uint32_t)(reinterpret_cast<uintptr_t>(f + pos) - win.base));
        const uint32_t hlen = ZDB_ENTRY_HEADER_SIZE + h.idl;
        if (pos + hlen > len) {
            st = ZDB_WALK_SHORT_HEADER;
            break;
        }
        const uint32_t L = h.L;
        uint64_t next = pos + hlen;
        int32_t s = ST_CONTINUE;
        if (L) {
            if (next + L > len)
                s = ZDB_WALK_SHORT_PAYLOAD;
            else
                next += L;
        }
        // the next window's loads are issued before the slot store (the
        // memory counter completes in order) and staged after it
        const bool reload = s == ST_CONTINUE && next < len && next < cend &&
                            reinterpret_cast<uintptr_t>(f + next) - win.base + 13u > WB;
        if (reload) {
            load_wide<WB>(win, f, len, next, lane);
            loads++;
        }
        __asm__ volatile("" ::: "memory");
        if (count < kcap && lane == 0) {
            const bool full = s == ST_CONTINUE && L > 0;
            sl[count] = RecSlot{(uint32_t)pos, full ? L : 0u, full ? h.integ : 0u, hlen};
        }
        count++;
        if (s == ZDB_WALK_SHORT_PAYLOAD) {
            st = s;
            break;
        }
        if (reload)
            stage_wide<WB>(win, lds, lane);
        pos = next;
    }
    if (st == ST_CONTINUE && pos >= len)
        st = ZDB_WALK_OK;
    if (lane == 0) {
        s_exit[w] = pos;
        s_count[w] = count;
        s_status[w] = st;
    }
    return loads;
}

__global__ __launch_bounds__(64) void walk_spec_win_kernel(FileTab t, const uint64_t *__restrict__ s_start,
                                                           uint64_t *__restrict__ s_exit,
                                                           uint32_t *__restrict__ s_count,
                                                           int32_t *__restrict__ s_status, RecSlot *__restrict__ slots,
                                                           uint32_t kcap) {
    const uint64_t start = s_start[blockIdx.x];
    if (start != NONE)
        chain_window(t, blockIdx.x, start, threadIdx.x, s_exit, s_count, s_status, slots, kcap);
}

// A1 + A2 in one kernel: the first wave of a chunk's search workgroup follows
// the chunk's chain as soon as its start is known, so the chains' round trips
// overlap the searches of the other chunks (and the next workgroups' start)
// instead of following all of them
// STAMP (diagnostic library): per chunk, s_memrealtime (100 MHz) at the
// start, after the search and after the chain, and the chain's window loads
template <int NT, int SU, int MW, uint32_t WB = 0, bool STAMP = false, bool ILP = SEARCH_ILP>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(MW))) void walk_search_chain_kernel(
    FileTab t, uint64_t *__restrict__ s_start, int32_t *__restrict__ s_status, uint64_t *__restrict__ s_exit,
    uint32_t *__restrict__ s_count, RecSlot *__restrict__ slots, uint32_t kcap, uint64_t *__restrict__ stamps) {
    const uint64_t t0 = STAMP ? __builtin_amdgcn_s_memrealtime() : 0;
    uint64_t start;
    int32_t status;
    search_chunk<NT, SU, true, ILP>(t, blockIdx.x, start, status);
    if (threadIdx.x == 0) {
        s_start[blockIdx.x] = start;
        s_status[blockIdx.x] = status;
    }
    if (threadIdx.x < 64) {
        const uint64_t t1 = STAMP ? __builtin_amdgcn_s_memrealtime() : 0;
        uint32_t loads = 0;
        if (start != NONE) {
            if (WB)
                loads = chain_wide<WB ? WB : 1024>(t, blockIdx.x, start, threadIdx.x, s_exit, s_count, s_status,
                                                   slots, kcap);
            else
                loads = chain_window(t, blockIdx.x, start, threadIdx.x, s_exit, s_count, s_status, slots, kcap);
        }
        if (STAMP && threadIdx.x == 0) {
            const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
            uint64_t *sp = stamps + 4 * (uint64_t)blockIdx.x;
            sp[0] = t0;
            sp[1] = t1;
            sp[2] = t2;
            sp[3] = loads;
        }
    }
}

enum ChunkMode : uint32_t { MODE_NONE = 0, MODE_COPY = 1, MODE_WALK = 2 };

// B: exact stitch (one thread per file); re-walks a chunk serially when its
// speculative start is not the true exit of the chunk before it
// the exact stitch of one file (see walk_stitch_kernel)
__device__ __forceinline__ void stitch_file(const FileTab &t, uint32_t fi, const uint64_t *__restrict__ s_start,
                                            const uint64_t *__restrict__ s_exit, const uint32_t *__restrict__ s_count,
                                            const int32_t *__restrict__ s_status, uint64_t *__restrict__ true_start,
                                            uint64_t *__restrict__ chunk_base, uint32_t *__restrict__ chunk_mode,
                                            uint32_t kcap, uint64_t *__restrict__ file_records,
                                            int32_t *__restrict__ file_status, uint32_t *__restrict__ rewalks) {
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
        const uint64_t cend = chunk_edge(t, fi, (uint64_t)c + 1);
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

#ifdef ZDBCRC_DIAG // the round-2 stitch (one thread per file), for A/B
__global__ __launch_bounds__(WALK_T) void walk_stitch_kernel(FileTab t, const uint64_t *__restrict__ s_start,
                                                             const uint64_t *__restrict__ s_exit,
                                                             const uint32_t *__restrict__ s_count,
                                                             const int32_t *__restrict__ s_status,
                                                             uint64_t *__restrict__ true_start,
                                                             uint64_t *__restrict__ chunk_base,
                                                             uint32_t *__restrict__ chunk_mode, uint32_t kcap,
                                                             uint64_t *__restrict__ file_records,
                                                             int32_t *__restrict__ file_status,
                                                             uint32_t *__restrict__ rewalks, bool prefix) {
    const uint32_t fi = blockIdx.x * WALK_T + threadIdx.x;
    if (fi < t.nfiles)
        stitch_file(t, fi, s_start, s_exit, s_count, s_status, true_start, chunk_base, chunk_mode, kcap, file_records,
                    file_status, rewalks);
    if (prefix) { // one block holds every file: the file prefix here instead of walk_prefix_kernel
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t acc = 0;
            uint32_t redo = 0;
            for (uint32_t i = 0; i < t.nfiles; i++) {
                const uint64_t n = file_records[i];
                file_records[i] = acc;
                acc += n;
                redo += rewalks[i];
            }
            file_records[t.nfiles] = acc;
            rewalks[t.nfiles] = redo;
        }
    }
}

#endif

// B, one wave per file: every chunk's speculative result checked at once
// (lane = chunk, 64 at a time).  The position that reaches chunk c is the
// exit of the nearest chunk below it with a speculative start, or the
// datafile header for chunk 0; the file is consistent when every live chunk
// either starts exactly there or has no start and is reached at or past its
// end (chunks after the first whose chain ended -- a terminal status -- are
// dead, as in the serial stitch).  Consistent files (zdbd's, always, unless
// one entry spans a chunk the search then mis-reads) get their chunk bases
// from a wave prefix sum; any other file is stitched serially by lane 0
// (stitch_file: the same outputs, by construction the reference order).
__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, (int)src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src, 64);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((uint32_t)v, l);
}

__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v, uint32_t lane) {
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint64_t u = shfl64(v, lane >= o ? lane - o : lane);
        v += lane >= o ? u : 0;
    }
    return v;
}

__device__ __forceinline__ void stitch_file_wave(const FileTab &t, uint32_t fi, uint32_t lane,
                                                 const uint64_t *__restrict__ s_start,
                                                 const uint64_t *__restrict__ s_exit,
                                                 const uint32_t *__restrict__ s_count,
                                                 const int32_t *__restrict__ s_status, uint64_t *__restrict__ true_start,
                                                 uint64_t *__restrict__ chunk_base, uint32_t *__restrict__ chunk_mode,
                                                 uint32_t kcap, uint64_t *__restrict__ file_records,
                                                 int32_t *__restrict__ file_status, uint32_t *__restrict__ rewalks) {
    const uint64_t len = t.file_len[fi];
    const uint64_t w0 = (uint64_t)fi * t.cpf;
    bool ok = len <= ((uint64_t)t.cpf << t.lg) && s_status[w0] != ZDB_WALK_BAD_DESCRIPTOR;
    uint64_t carry_pos = ZDB_DATA_HEADER_SIZE, total = 0;
    bool carry_dead = false;
    int32_t fst = ST_CONTINUE;
    const uint64_t below_mask = (1ull << lane) - 1; // lanes under this one (lane 0: none)
    for (uint32_t g = 0; ok && g < t.cpf; g += 64) {
        const uint32_t c = g + lane;
        const bool in = c < t.cpf;
        const uint64_t w = w0 + c;
        const uint64_t ss = in ? s_start[w] : NONE;
        const bool act = ss != NONE;
        const uint64_t ex = act ? s_exit[w] : 0;
        const uint32_t cnt = act ? s_count[w] : 0u;
        const int32_t cs = act ? s_status[w] : ST_CONTINUE;
        const uint64_t am = __ballot(act);
        const uint64_t tm = __ballot(act && cs != ST_CONTINUE);
        const uint64_t below = am & below_mask;
        const uint64_t pb_in = shfl64(ex, below ? 63u - (uint32_t)__clzll(below) : lane);
        const uint64_t pb = below ? pb_in : carry_pos;
        const bool dead = carry_dead || (tm & below_mask) != 0;
        const uint64_t cend = chunk_edge(t, fi, (uint64_t)c + 1);
        const bool good = !in || dead || (act ? ss == pb : pb >= cend);
        if (__ballot(!good)) {
            ok = false;
            break;
        }
        const bool walked = in && !dead && act;
        const uint64_t v = walked ? cnt : 0;
        const uint64_t incl = wave_incl_scan64(v, lane);
        if (in) {
            chunk_base[w] = total + incl - v;
            true_start[w] = walked ? ss : NONE;
            chunk_mode[w] = walked ? (cnt <= kcap ? MODE_COPY : MODE_WALK) : MODE_NONE;
        }
        total += readlane64(incl, 63);
        const uint64_t twm = __ballot(walked && cs != ST_CONTINUE);
        if (twm && fst == ST_CONTINUE)
            fst = __builtin_amdgcn_readlane(cs, (uint32_t)__builtin_ctzll(twm));
        if (am)
            carry_pos = readlane64(ex, 63u - (uint32_t)__clzll(am));
        carry_dead = carry_dead || tm != 0;
    }
    if (!ok) { // rewrites every output of the file (same wave: the stores above land first)
        if (lane == 0)
            stitch_file(t, fi, s_start, s_exit, s_count, s_status, true_start, chunk_base, chunk_mode, kcap,
                        file_records, file_status, rewalks);
        return;
    }
    if (lane == 0) {
        file_records[fi] = total;
        file_status[fi] = fst == ST_CONTINUE ? ZDB_WALK_OK : fst;
        rewalks[fi] = 0;
    }
}

// one wave per file; the last wave to finish (ticket counter, reset by it)
// turns the per-file counts into the exclusive file prefix (entry nfiles =
// total) and sums the re-walks, 64 files per step
__global__ __launch_bounds__(64) void walk_stitch_wave_kernel(
    FileTab t, const uint64_t *__restrict__ s_start, const uint64_t *__restrict__ s_exit,
    const uint32_t *__restrict__ s_count, const int32_t *__restrict__ s_status, uint64_t *__restrict__ true_start,
    uint64_t *__restrict__ chunk_base, uint32_t *__restrict__ chunk_mode, uint32_t kcap,
    uint64_t *__restrict__ file_records, int32_t *__restrict__ file_status, uint32_t *__restrict__ rewalks,
    uint32_t *__restrict__ done) {
    const uint32_t lane = threadIdx.x;
    stitch_file_wave(t, blockIdx.x, lane, s_start, s_exit, s_count, s_status, true_start, chunk_base, chunk_mode,
                     kcap, file_records, file_status, rewalks);
    __threadfence(); // this file's counts are visible device-wide before its ticket
    uint32_t ticket = 0;
    if (lane == 0)
        ticket = atomicAdd(done, 1u);
    ticket = (uint32_t)__shfl((int)ticket, 0, 64);
    if (ticket != t.nfiles - 1)
        return;
    __threadfence(); // every other file's counts are visible here
    uint64_t acc = 0;
    uint32_t redo = 0;
    for (uint32_t b = 0; b < t.nfiles; b += 64) {
        const uint32_t i = b + lane;
        const uint64_t n = i < t.nfiles ? file_records[i] : 0;
        const uint32_t r = i < t.nfiles ? rewalks[i] : 0u;
        const uint64_t incl = wave_incl_scan64(n, lane);
        if (i < t.nfiles)
            file_records[i] = acc + incl - n;
        acc += readlane64(incl, 63);
        redo += (uint32_t)readlane64(wave_incl_scan64(r, lane), 63);
    }
    if (lane == 0) {
        file_records[t.nfiles] = acc;
        rewalks[t.nfiles] = redo;
        *done = 0; // for the next walk on this workspace (stream order)
    }
}

#ifdef ZDBCRC_DIAG
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
#endif

// C1: descriptors of the accepted chunks, copied from their slots (one
// thread per slot)
// slot g of the accepted chunks -> its final descriptor (C1)
__device__ __forceinline__ void copy_slot(const FileTab &t, uint64_t g, const uint32_t *__restrict__ chunk_mode,
                                          const uint32_t *__restrict__ s_count, const RecSlot *__restrict__ slots,
                                          uint32_t kcap, const uint64_t *__restrict__ chunk_base,
                                          const uint64_t *__restrict__ file_base, uint64_t capacity,
                                          uint64_t *__restrict__ entry_off, uint64_t *__restrict__ poff,
                                          uint32_t *__restrict__ plen, uint32_t *__restrict__ expect) {
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
// records than slots (one lane per chunk, CHAINS_PER_WAVE per one-wave
// workgroup, as A2)
// chunk w, when it was re-walked or overflowed its slots: a serial walk
// writes its descriptors (C2)
__device__ __forceinline__ void emit_chunk(const FileTab &t, uint64_t w, const uint64_t *__restrict__ true_start,
                                           const uint32_t *__restrict__ chunk_mode,
                                           const uint64_t *__restrict__ chunk_base,
                                           const uint64_t *__restrict__ file_base, uint64_t capacity,
                                           uint64_t *__restrict__ entry_off, uint64_t *__restrict__ poff,
                                           uint32_t *__restrict__ plen, uint32_t *__restrict__ expect) {
    if (w >= (uint64_t)t.nfiles * t.cpf || chunk_mode[w] != MODE_WALK)
        return;
    const uint32_t fi = (uint32_t)(w / t.cpf), c = (uint32_t)(w % t.cpf);
    const uint64_t cend = chunk_edge(t, fi, (uint64_t)c + 1);
    const uint64_t foff = t.file_off[fi];
    uint32_t count;
    uint64_t exit;
    int32_t st;
    walk_chain<EMIT>(t.image + foff, t.file_len[fi], true_start[w], cend, count, exit, st, nullptr, 0, foff,
                     file_base[fi] + chunk_base[w], capacity, entry_off, poff, plen, expect);
}

// C1 + C2 in one launch: blocks [0, ncopy) copy the slots of accepted chunks,
// the blocks after them emit the re-walked ones (one chunk per thread; rare)
__global__ __launch_bounds__(WALK_T) void walk_out_kernel(FileTab t, const uint64_t *__restrict__ true_start,
                                                          const uint32_t *__restrict__ chunk_mode,
                                                          const uint32_t *__restrict__ s_count,
                                                          const RecSlot *__restrict__ slots, uint32_t kcap,
                                                          const uint64_t *__restrict__ chunk_base,
                                                          const uint64_t *__restrict__ file_base, uint64_t capacity,
                                                          uint64_t *__restrict__ entry_off, uint64_t *__restrict__ poff,
                                                          uint32_t *__restrict__ plen, uint32_t *__restrict__ expect,
                                                          uint32_t ncopy) {
    if (blockIdx.x < ncopy)
        copy_slot(t, (uint64_t)blockIdx.x * WALK_T + threadIdx.x, chunk_mode, s_count, slots, kcap, chunk_base,
                  file_base, capacity, entry_off, poff, plen, expect);
    else
        emit_chunk(t, (uint64_t)(blockIdx.x - ncopy) * WALK_T + threadIdx.x, true_start, chunk_mode, chunk_base,
                   file_base, capacity, entry_off, poff, plen, expect);
}

#ifdef ZDBCRC_DIAG
struct LastWalk {
    uint8_t *ws;
    uint64_t nchunks;
} g_last_walk = {nullptr, 0};

uint32_t chains_per_wave() { // A/B: ZDBCRC_CHAINS_PER_WAVE (1..64)
    static const uint32_t v = [] {
        const char *e = std::getenv("ZDBCRC_CHAINS_PER_WAVE");
        const int x = e ? std::atoi(e) : 0;
        return x >= 1 && x <= 64 ? (uint32_t)x : CHAINS_PER_WAVE;
    }();
    return v;
}

int chain_mode() { // A/B: ZDBCRC_CHAIN_MODE (0: one lane per chunk, 1: one wave per chunk, 1 KiB windows,
                   // 2: the windowed chain fused into the search kernel)
    static const int v = [] {
        const char *e = std::getenv("ZDBCRC_CHAIN_MODE");
        return e ? std::atoi(e) : -1;
    }();
    return v;
}

// A/B: ZDBCRC_CHAIN_WB or zdbcrc_debug_set_chain_wb (0: 1 KiB register
// window, else LDS window bytes)
int g_chain_wb = -1;
uint64_t *g_stamps = nullptr;
uint64_t g_stamps_n = 0, g_stamps_used = 0;
uint32_t chain_wb() {
    if (g_chain_wb < 0) {
        const char *e = std::getenv("ZDBCRC_CHAIN_WB");
        g_chain_wb = e ? std::atoi(e) : (int)CHAIN_WB;
    }
    return (uint32_t)g_chain_wb;
}

bool search_ilp() { // A/B: ZDBCRC_SEARCH_ILP=0/1 (the fused walk's search filter shape)
    static const bool v = [] {
        const char *e = std::getenv("ZDBCRC_SEARCH_ILP");
        return e ? std::atoi(e) == 1 : SEARCH_ILP;
    }();
    return v;
}

int search_nt() { // A/B: ZDBCRC_SEARCH_NT = 512 / 1024 threads per chunk in the fused walk
    static const int v = [] {
        const char *e = std::getenv("ZDBCRC_SEARCH_NT");
        return e ? std::atoi(e) : SEARCH_T;
    }();
    return v;
}

int search_ilp_mw() {
    static const int v = [] {
        const char *e = std::getenv("ZDBCRC_SEARCH_ILP_MW");
        return e ? std::atoi(e) : 6;
    }();
    return v;
}

bool chunk_skew() { // A/B: ZDBCRC_CHUNK_SKEW=0/1
    static const bool v = [] {
        const char *e = std::getenv("ZDBCRC_CHUNK_SKEW");
        return e ? std::atoi(e) == 1 : CHUNK_SKEW;
    }();
    return v;
}

bool serial_stitch() { // A/B: ZDBCRC_SERIAL_STITCH=1 -> one thread per file (the round-2 stitch)
    static const bool v = [] {
        const char *e = std::getenv("ZDBCRC_SERIAL_STITCH");
        return e && std::atoi(e) == 1;
    }();
    return v;
}

int search_variant() {
    static const int v = [] {
        const char *e = std::getenv("ZDBCRC_SEARCH_VARIANT");
        return e ? std::atoi(e) : 0;
    }();
    return v;
}
#endif

#ifdef ZDBCRC_DIAG
// search-rate probe: every wave scans its own bytes_per_wave of the image
// with the search filter, no early exit and no barrier (MODE 0: scan_block
// backward shape, full filter + confirmation; 1: the same loads, no filter;
// 2: scan_block_ilp; 3: MODE 0 + a workgroup barrier per block, as the search
// loop has)
template <int MODE, int SU>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void search_rate_kernel(
    const uint8_t *__restrict__ img, uint64_t len, uint64_t per_wave, uint32_t *__restrict__ sink) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t b0 = 4096 + w * per_wave;
    // positions relative to a 256 MiB "file" (the search's `previous` < p
    // test passes as often as in C4's files)
    const uint64_t fb = b0 & ~((1ull << 28) - 1);
    const uint8_t *f = img + fb;
    uint32_t x = 0;
    for (uint64_t b = b0; b < b0 + per_wave && b + 1024u * SU + 64 < len; b += 1024u * SU) {
        if (MODE == 1) {
            uint4 v[SU];
#pragma unroll
            for (int u = 0; u < SU; u++)
                v[u] = *reinterpret_cast<const uint4 *>(img + b + 1024u * u + 16u * lane);
#pragma unroll
            for (int u = 0; u < SU; u++)
                x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        } else if (MODE == 2) {
            x ^= (uint32_t)scan_block_ilp<false, SU>(f, len - fb, b - fb, 28, len - fb, lane);
        } else if (MODE == 5) { // the other filter shape
            x ^= (uint32_t)scan_block<false, SU, true, false, !FILTER_OR>(f, len - fb, b - fb, 28, len - fb, lane);
        } else {
            x ^= (uint32_t)scan_block<false, SU, true>(f, len - fb, b - fb, 28, len - fb, lane);
            if (MODE == 3)
                __syncthreads();
        }
    }
    if (x == 0x12345678u)
        sink[0] = x;
}

// zdbcrc_debug_search_rate: ms of one probe launch over grid workgroups
float search_rate_ms(const uint8_t *d_img, uint64_t len, int mode, uint64_t per_wave, uint32_t grid) {
    static uint32_t *sink = nullptr;
    if (!sink && hipMalloc(&sink, 64) != hipSuccess)
        return -1.f;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    switch (mode) {
    case 0: hipLaunchKernelGGL((search_rate_kernel<0, 8>), dim3(grid), dim3(256), 0, 0, d_img, len, per_wave, sink); break;
    case 1: hipLaunchKernelGGL((search_rate_kernel<1, 8>), dim3(grid), dim3(256), 0, 0, d_img, len, per_wave, sink); break;
    case 2: hipLaunchKernelGGL((search_rate_kernel<2, 8>), dim3(grid), dim3(256), 0, 0, d_img, len, per_wave, sink); break;
    case 3: hipLaunchKernelGGL((search_rate_kernel<3, 8>), dim3(grid), dim3(256), 0, 0, d_img, len, per_wave, sink); break;
    case 4: hipLaunchKernelGGL((search_rate_kernel<0, 4>), dim3(grid), dim3(256), 0, 0, d_img, len, per_wave, sink); break;
    case 5: hipLaunchKernelGGL((search_rate_kernel<5, 8>), dim3(grid), dim3(256), 0, 0, d_img, len, per_wave, sink); break;
    default: return -1.f;
    }
    hipEventRecord(e1, 0);
    float ms = -1.f;
    if (hipEventSynchronize(e1) == hipSuccess)
        hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return ms;
}
#endif

// default chunk size, from the record density of the store: one wave per
// file walks the headers of its first DENSITY_SAMPLE bytes through 4 KiB LDS
// windows (records that start there, and the bytes they cover, summed over
// the files).  A chunk's chain has one dependent round trip per record that
// does not share a window with the one before it, so a store of small values
// (4 KiB: ~2,000 records per 8 MiB chunk) needs smaller chunks, while C4's
// Zipf mix (~170 records per 8 MiB, most bytes in long values that every
// chunk start has to search across) needs large ones.
constexpr uint32_t DENSITY_SAMPLE = 64u << 10;
constexpr uint32_t DENSITY_MAX_PER_CHUNK = 512; // records per default chunk before it is made smaller
constexpr uint32_t DENSITY_TARGET = 128;        // records per chunk when it is
constexpr uint32_t MIN_LG_CHUNK = 16;
// a store whose default chunks outnumber the search workgroups the GPU holds
// at once (6 per CU at <= 80 VGPRs) walks in chunks twice as large, when its
// density keeps them within half their slots: the last chunks no longer wait
// 100-170 us for a free slot (C4: 2,048 chunks, 1,536 resident; stamped
// span 440 -> 391 us, profiles/r3/walk_width_chunk.jsonl)
constexpr uint32_t SEARCH_WG_PER_CU = 6;
constexpr uint32_t LARGE_LG_CHUNK = 24;
// record slots per chunk (beyond them a chunk's records are emitted by a
// serial re-walk): 512, 1,024 for the large chunks
__host__ __device__ constexpr uint32_t chunk_slots(uint32_t lg, uint64_t nchunks) {
    return nchunks > 65536 ? 64u : lg >= LARGE_LG_CHUNK ? 1024u : 512u;
}

__global__ __launch_bounds__(64) void walk_density_kernel(FileTab t, unsigned long long *__restrict__ acc) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[4096 / 4 + 4];
    const uint32_t fi = blockIdx.x, lane = threadIdx.x;
    const uint64_t len = t.file_len[fi];
    const uint8_t *f = t.image + t.file_off[fi];
    const uint64_t lim = len < DENSITY_SAMPLE + ZDB_DATA_HEADER_SIZE ? len : DENSITY_SAMPLE + ZDB_DATA_HEADER_SIZE;
    uint64_t pos = ZDB_DATA_HEADER_SIZE;
    uint32_t count = 0;
    WideWindow<4096> win;
    win.base = 0;
    bool have = false;
    while (pos < lim && pos + ZDB_ENTRY_HEADER_SIZE <= len) {
        if (!have || reinterpret_cast<uintptr_t>(f + pos) - win.base + 13u > 4096u) {
            load_wide<4096>(win, f, len, pos, lane);
            stage_wide<4096>(win, lds, lane);
            have = true;
        }
        const Hdr h = lds_hdr(lds, (uint32_t)(reinterpret_cast<uintptr_t>(f + pos) - win.base));
        const uint64_t next = pos + ZDB_ENTRY_HEADER_SIZE + h.idl + h.L;
        if (next > len)
            break;
        count++;
        pos = next;
    }
    if (lane == 0 && count) {
        atomicAdd(acc, (unsigned long long)count);
        atomicAdd(acc + 1, (unsigned long long)(pos - ZDB_DATA_HEADER_SIZE));
    }
}

struct DensityKey {
    const uint8_t *image;
    const uint64_t *file_off;
    uint32_t nfiles;
    uint64_t max_file_len;
    bool operator<(const DensityKey &o) const {
        return std::tie(image, file_off, nfiles, max_file_len) < std::tie(o.image, o.file_off, o.nfiles, o.max_file_len);
    }
};

// per (device, stream) workspace of the walk
struct WalkWs {
    void *ptr = nullptr;
    size_t bytes = 0;
};
std::mutex g_walk_mu[64];
std::map<void *, WalkWs> g_walk_ws[64];
// the default chunk size chosen for a store, by its image and file table
// (any chunk size gives the same walk: a stale entry after the same buffers
// are refilled with another store only costs time)
std::map<DensityKey, uint32_t> g_walk_lg[64];
unsigned long long *g_density_acc[64];

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
    zdbcrc_internal_mark_hip();
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64)
        return ZDB_CRC32_ENODEV;
    hipStream_t st = static_cast<hipStream_t>(stream);
    std::lock_guard<std::mutex> g(g_walk_mu[dev]);
    if (!chunk_bytes) { // the store's own default (walk_density_kernel), measured once per store
        const DensityKey key{d_image, d_file_off, nfiles, max_file_len};
        auto it = g_walk_lg[dev].find(key);
        if (it != g_walk_lg[dev].end()) {
            lg = it->second;
        } else {
            if (!g_density_acc[dev] && hipMalloc(&g_density_acc[dev], 2 * sizeof(unsigned long long)) != hipSuccess)
                return ZDB_CRC32_ENOMEM;
            unsigned long long h[2] = {0, 0};
            const FileTab t0{d_image, d_file_off, d_file_len, nfiles, 1, DEFAULT_LG_CHUNK, 0};
            if (hipMemsetAsync(g_density_acc[dev], 0, sizeof(h), st) != hipSuccess)
                return ZDB_CRC32_ELAUNCH;
            hipLaunchKernelGGL(walk_density_kernel, dim3(nfiles), dim3(64), 0, st, t0, g_density_acc[dev]);
            if (hipGetLastError() != hipSuccess ||
                hipMemcpyAsync(h, g_density_acc[dev], sizeof(h), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess)
                return ZDB_CRC32_ELAUNCH;
            // records per default chunk = count / bytes * 2^23
            if (h[0] && h[1] && (double)h[0] * (double)(1ull << DEFAULT_LG_CHUNK) >
                                     (double)DENSITY_MAX_PER_CHUNK * (double)h[1]) {
                const double c = (double)DENSITY_TARGET * (double)h[1] / (double)h[0]; // bytes per target chunk
                while (lg > MIN_LG_CHUNK && (double)(1ull << lg) > c)
                    lg--;
            } else if (h[0] && h[1]) {
                int cus = 0;
                const uint64_t n8 = (max_file_len + (1ull << DEFAULT_LG_CHUNK) - 1) >> DEFAULT_LG_CHUNK;
                if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                    cus > 0 && n8 * nfiles > (uint64_t)cus * SEARCH_WG_PER_CU &&
                    (double)h[0] * (double)(1ull << LARGE_LG_CHUNK) <=
                        0.5 * chunk_slots(LARGE_LG_CHUNK, 1) * (double)h[1])
                    lg = LARGE_LG_CHUNK;
            }
            g_walk_lg[dev][key] = lg;
        }
    }
    const uint64_t cpf64 = max_file_len ? (max_file_len + (1ull << lg) - 1) >> lg : 1;
    const uint64_t nchunks = cpf64 * nfiles;
    // one search workgroup of SEARCH_T threads per chunk and up to 512 slot
    // threads per chunk in the copy: keep every grid below 2^32 threads, so
    // an oversized store fails here and not as a late launch error
    const uint32_t kcap = chunk_slots(lg, nchunks);
    if (nchunks >= (1ull << 32) / SEARCH_T || nchunks * kcap >= (1ull << 32))
        return ZDB_CRC32_EINVAL;
    // workspace: per chunk s_start, s_exit, true_start, chunk_base (u64),
    // s_count, s_status, chunk_mode (4 B), kcap record slots (16 B each)
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    // (+ the stitch's ticket counter, zero between walks)
    const size_t need = 4 * al(nchunks * 8) + 3 * al(nchunks * 4) + al(nchunks * kcap * sizeof(RecSlot)) + 256;
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
        if (hipMemsetAsync(static_cast<uint8_t *>(ws.ptr) + need - 256, 0, 256, st) != hipSuccess)
            return ZDB_CRC32_ELAUNCH;
    }
    uint8_t *b = static_cast<uint8_t *>(ws.ptr);
#ifdef ZDBCRC_DIAG
    g_last_walk = {b, nchunks};
#endif
    uint64_t *s_start = reinterpret_cast<uint64_t *>(b);
    uint64_t *s_exit = reinterpret_cast<uint64_t *>(b + al(nchunks * 8));
    uint64_t *true_start = reinterpret_cast<uint64_t *>(b + 2 * al(nchunks * 8));
    uint64_t *chunk_base = reinterpret_cast<uint64_t *>(b + 3 * al(nchunks * 8));
    uint32_t *s_count = reinterpret_cast<uint32_t *>(b + 4 * al(nchunks * 8));
    int32_t *s_status = reinterpret_cast<int32_t *>(b + 4 * al(nchunks * 8) + al(nchunks * 4));
    uint32_t *chunk_mode = reinterpret_cast<uint32_t *>(b + 4 * al(nchunks * 8) + 2 * al(nchunks * 4));
    RecSlot *slots = reinterpret_cast<RecSlot *>(b + 4 * al(nchunks * 8) + 3 * al(nchunks * 4));
    uint32_t *done = reinterpret_cast<uint32_t *>(b + ws.bytes - 256);

#ifdef ZDBCRC_DIAG
    const FileTab t{d_image, d_file_off, d_file_len, nfiles, (uint32_t)cpf64, lg, chunk_skew() ? 1u : 0u};
#else
    const FileTab t{d_image, d_file_off, d_file_len, nfiles, (uint32_t)cpf64, lg, CHUNK_SKEW ? 1u : 0u};
#endif
#ifdef ZDBCRC_DIAG
    const uint32_t cpw = chains_per_wave();
#else
    const uint32_t cpw = CHAINS_PER_WAVE;
#endif
    const dim3 gchain((uint32_t)((nchunks + cpw - 1) / cpw));
#ifdef ZDBCRC_DIAG
    const bool fused = chain_mode() >= 0 ? chain_mode() == 2 : FUSED_WALK;
#else
    const bool fused = FUSED_WALK;
#endif
#ifdef ZDBCRC_DIAG
    const uint32_t wb = chain_wb();
#else
    constexpr uint32_t wb = CHAIN_WB;
#endif
    if (fused) {
#define ZDBCRC_FUSED(WBV)                                                                                              \
    hipLaunchKernelGGL((walk_search_chain_kernel<SEARCH_T, SEARCH_SU, SEARCH_MW, WBV>), dim3((uint32_t)nchunks),       \
                       dim3(SEARCH_T), 0, st, t, s_start, s_status, s_exit, s_count, slots, kcap, nullptr)
#ifdef ZDBCRC_DIAG
#define ZDBCRC_FUSED_STAMP(WBV)                                                                                        \
    hipLaunchKernelGGL((walk_search_chain_kernel<SEARCH_T, SEARCH_SU, SEARCH_MW, WBV, true>),                          \
                       dim3((uint32_t)nchunks), dim3(SEARCH_T), 0, st, t, s_start, s_status, s_exit, s_count, slots,   \
                       kcap, g_stamps)
        if (search_nt() == 384 || search_nt() == 512 || search_nt() == 768 || search_nt() == 1024) {
            // A/B: more waves per chunk search
            const bool stamp = g_stamps && nchunks <= g_stamps_n;
            if (stamp)
                g_stamps_used = nchunks;
            uint64_t *sp = stamp ? g_stamps : nullptr;
#define ZDBCRC_NT(N)                                                                                                   \
    if (search_nt() == N) {                                                                                            \
        if (stamp)                                                                                                     \
            hipLaunchKernelGGL((walk_search_chain_kernel<N, SEARCH_SU, SEARCH_MW, 2048, true>), dim3((uint32_t)nchunks), \
                               dim3(N), 0, st, t, s_start, s_status, s_exit, s_count, slots, kcap, sp);                \
        else                                                                                                           \
            hipLaunchKernelGGL((walk_search_chain_kernel<N, SEARCH_SU, SEARCH_MW, 2048, false>), dim3((uint32_t)nchunks), \
                               dim3(N), 0, st, t, s_start, s_status, s_exit, s_count, slots, kcap, sp);                \
    }
            ZDBCRC_NT(384)
            ZDBCRC_NT(512)
            ZDBCRC_NT(768)
            ZDBCRC_NT(1024)
#undef ZDBCRC_NT
        } else if (search_ilp() != SEARCH_ILP) {
            if (search_ilp_mw() == 5)
                hipLaunchKernelGGL((walk_search_chain_kernel<SEARCH_T, SEARCH_SU, 5, 0, false, !SEARCH_ILP>),
                                   dim3((uint32_t)nchunks), dim3(SEARCH_T), 0, st, t, s_start, s_status, s_exit,
                                   s_count, slots, kcap, nullptr);
            else if (wb == 2048)
                hipLaunchKernelGGL((walk_search_chain_kernel<SEARCH_T, SEARCH_SU, SEARCH_MW, 2048, false, !SEARCH_ILP>),
                                   dim3((uint32_t)nchunks), dim3(SEARCH_T), 0, st, t, s_start, s_status, s_exit,
                                   s_count, slots, kcap, nullptr);
            else
                hipLaunchKernelGGL((walk_search_chain_kernel<SEARCH_T, SEARCH_SU, SEARCH_MW, 0, false, !SEARCH_ILP>),
                                   dim3((uint32_t)nchunks), dim3(SEARCH_T), 0, st, t, s_start, s_status, s_exit,
                                   s_count, slots, kcap, nullptr);
        } else if (g_stamps && nchunks <= g_stamps_n) {
            g_stamps_used = nchunks;
            if (wb == 2048)
                ZDBCRC_FUSED_STAMP(2048);
            else
                ZDBCRC_FUSED_STAMP(0);
        } else
#undef ZDBCRC_FUSED_STAMP
#endif
        switch (wb) {
#ifdef ZDBCRC_DIAG
        case 1024: ZDBCRC_FUSED(1024); break;
        case 4096: ZDBCRC_FUSED(4096); break;
        case 8192: ZDBCRC_FUSED(8192); break;
#endif
        case 2048: ZDBCRC_FUSED(2048); break;
        default: ZDBCRC_FUSED(0); break;
        }
#undef ZDBCRC_FUSED
    } else {
#ifdef ZDBCRC_DIAG
    switch (search_variant()) { // A/B (scripts/walk_probe.py with the diagnostic library)
    case 9: hipLaunchKernelGGL((walk_search_kernel<256, 8, false>), dim3((uint32_t)nchunks), dim3(256), 0, st, t, s_start, s_status); break;
    case 1: hipLaunchKernelGGL((walk_search_kernel<128, 8>), dim3((uint32_t)nchunks), dim3(128), 0, st, t, s_start, s_status); break;
    case 2: hipLaunchKernelGGL((walk_search_kernel<256, 16>), dim3((uint32_t)nchunks), dim3(256), 0, st, t, s_start, s_status); break;
    case 3: hipLaunchKernelGGL((walk_search_kernel<512, 8>), dim3((uint32_t)nchunks), dim3(512), 0, st, t, s_start, s_status); break;
    case 4: hipLaunchKernelGGL((walk_search_kernel<128, 16>), dim3((uint32_t)nchunks), dim3(128), 0, st, t, s_start, s_status); break;
    case 5: hipLaunchKernelGGL((walk_search_kernel<512, 4>), dim3((uint32_t)nchunks), dim3(512), 0, st, t, s_start, s_status); break;
    case 6: hipLaunchKernelGGL((walk_search_kernel<256, 8, true>), dim3((uint32_t)nchunks), dim3(256), 0, st, t, s_start, s_status); break;
    case 7: hipLaunchKernelGGL((walk_search_kernel<256, 16, true>), dim3((uint32_t)nchunks), dim3(256), 0, st, t, s_start, s_status); break;
    case 8: hipLaunchKernelGGL((walk_search_kernel<128, 16, true>), dim3((uint32_t)nchunks), dim3(128), 0, st, t, s_start, s_status); break;
    // occupancy: at most 64 / 80 VGPRs (8 / 6 waves per SIMD; the default shape takes 82 -> 5)
    case 10: hipLaunchKernelGGL((walk_search_kernel<256, 8, true, 8>), dim3((uint32_t)nchunks), dim3(256), 0, st, t, s_start, s_status); break;
    case 11: hipLaunchKernelGGL((walk_search_kernel<256, 4, true, 8>), dim3((uint32_t)nchunks), dim3(256), 0, st, t, s_start, s_status); break;
    case 12: hipLaunchKernelGGL((walk_search_kernel<256, 8, true, 6>), dim3((uint32_t)nchunks), dim3(256), 0, st, t, s_start, s_status); break;
    case 13: hipLaunchKernelGGL((walk_search_kernel<128, 8, true, 8>), dim3((uint32_t)nchunks), dim3(128), 0, st, t, s_start, s_status); break;
    default:
#endif
    hipLaunchKernelGGL((walk_search_kernel<SEARCH_T, SEARCH_SU, true, SEARCH_MW>), dim3((uint32_t)nchunks), dim3(SEARCH_T), 0,
                       st, t, s_start, s_status);
#ifdef ZDBCRC_DIAG
    }
#endif
#ifdef ZDBCRC_DIAG
    const bool win_chain = chain_mode() >= 0 ? chain_mode() == 1 : WINDOW_CHAIN;
#else
    const bool win_chain = WINDOW_CHAIN;
#endif
    if (win_chain)
        hipLaunchKernelGGL(walk_spec_win_kernel, dim3((uint32_t)nchunks), dim3(64), 0, st, t, s_start, s_exit,
                           s_count, s_status, slots, kcap);
    else
        hipLaunchKernelGGL(walk_spec_kernel, gchain, dim3(64), 0, st, t, s_start, s_exit, s_count, s_status, slots,
                           kcap, cpw);
    } // not fused
#ifdef ZDBCRC_DIAG
    if (serial_stitch()) {
        const bool one_block = nfiles <= WALK_T; // stitch and file prefix in one launch
        hipLaunchKernelGGL(walk_stitch_kernel, dim3((nfiles + WALK_T - 1) / WALK_T), dim3(WALK_T), 0, st, t,
                           s_start, s_exit, s_count, s_status, true_start, chunk_base, chunk_mode, kcap,
                           d_file_records, d_file_status, d_rewalks, one_block);
        if (!one_block)
            hipLaunchKernelGGL(walk_prefix_kernel, dim3(1), dim3(64), 0, st, nfiles, d_file_records, d_rewalks);
    } else
#endif
    hipLaunchKernelGGL(walk_stitch_wave_kernel, dim3(nfiles), dim3(64), 0, st, t, s_start, s_exit, s_count,
                       s_status, true_start, chunk_base, chunk_mode, kcap, d_file_records, d_file_status, d_rewalks,
                       done);
    if (capacity) {
        const uint64_t ncopy = (nchunks * kcap + WALK_T - 1) / WALK_T, nemit = (nchunks + WALK_T - 1) / WALK_T;
        hipLaunchKernelGGL(walk_out_kernel, dim3((uint32_t)(ncopy + nemit)), dim3(WALK_T), 0, st, t, true_start,
                           chunk_mode, s_count, slots, kcap, chunk_base, d_file_records, capacity, d_entry_off,
                           d_payload_off, d_payload_len, d_expected, (uint32_t)ncopy);
    }
    return hipGetLastError() == hipSuccess ? ZDB_CRC32_OK : ZDB_CRC32_ELAUNCH;
}

#ifdef ZDBCRC_DIAG
// measurement/debug hook: the speculative and the true start of every chunk
// of the last walk (device arrays copied to host; NONE = ~0)
// measurement hook: stamp the next fused walks into a device buffer of n
// chunks x 4 u64 (see walk_search_chain_kernel); returns the chunks stamped
// by the last walk (0 to switch off: d_stamps == nullptr)
uint64_t zdbcrc_debug_walk_stamps(uint64_t *d_stamps, uint64_t n) {
    const uint64_t used = g_stamps_used;
    g_stamps = d_stamps;
    g_stamps_n = d_stamps ? n : 0;
    g_stamps_used = 0;
    return used;
}

float zdbcrc_debug_search_rate(const uint8_t *d_img, uint64_t len, int mode, uint64_t per_wave, uint32_t grid) {
    return search_rate_ms(d_img, len, mode, per_wave, grid);
}

// A/B hook: the chain window of the fused walk (0, 1024, 2048, 4096, 8192)
int zdbcrc_debug_set_chain_wb(int wb) {
    if (wb != 0 && wb != 1024 && wb != 2048 && wb != 4096 && wb != 8192)
        return -1;
    g_chain_wb = wb;
    return 0;
}

int zdbcrc_debug_walk_starts(uint64_t *s_start, uint64_t *true_start, uint64_t nchunks) {
    if (!g_last_walk.ws || nchunks != g_last_walk.nchunks)
        return -1;
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    const uint8_t *b = g_last_walk.ws;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(s_start, b, nchunks * 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(true_start, b + 2 * al(nchunks * 8), nchunks * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return 0;
}
#endif

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
    if (nfiles && !b->capacity) {
        // a size query: the walk ran and counted; nothing was checksummed
        uint64_t n = 0;
        if (hipMemsetAsync(b->mismatch_count, 0, sizeof(uint32_t), st) != hipSuccess ||
            hipMemcpyAsync(&n, b->file_records + nfiles, sizeof(n), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return ZDB_CRC32_ELAUNCH;
        *n_records = n;
        return n ? ZDB_CRC32_ENOSPC : ZDB_CRC32_OK;
    }
    if (!nfiles)
        return zdb_crc32_verify_device(d_image, b->payload_off, b->payload_len, b->expected, b->computed,
                                       b->mismatch, b->mismatch_count, b->max_mismatch, 0, stream);
    // the verify reads the walk's record count from device memory (bounded by
    // the capacity: a walk that found more records wrote only that many), so
    // no host round trip separates the two; the count comes back at the end
    const uint64_t bound = b->capacity < 0xFFFFFFFFull ? b->capacity : 0xFFFFFFFFull; // 32-bit record indices
    rc = zdbcrc_internal_verify_device_dn(d_image, b->payload_off, b->payload_len, b->expected, b->computed,
                                          b->mismatch, b->mismatch_count, b->max_mismatch, bound,
                                          b->file_records + nfiles, stream);
    if (rc)
        return rc;
    uint64_t n = 0;
    if (hipMemcpyAsync(&n, b->file_records + nfiles, sizeof(n), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return ZDB_CRC32_ELAUNCH;
    *n_records = n;
    if (n > b->capacity)
        return ZDB_CRC32_ENOSPC;
    return n > bound ? ZDB_CRC32_EINVAL : ZDB_CRC32_OK; // more records than 32-bit indices reach
}

} // extern "C"
