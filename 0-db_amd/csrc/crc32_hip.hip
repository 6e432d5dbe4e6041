// crc32_hip.hip -- MI355X (gfx950) batched record checksum for 0-db.
//
// Computes out[r] = zdb_crc32(arena + offsets[r], lengths[r]) for n records
// in one pass over HBM (libzdb/crc32.c:145-155 semantics: CRC-32C, reflected
// 0x82F63B78, init 0, no final XOR).  Callers it serves: the SET path
// (commands_set.c:106/:216, api.c:124/:204), CHECK (data.c:564) and the
// integrity scan (integrity-check.c:90).
//
// Design (DESIGN.md §3 has the derivation and the roofline):
//  * The checksum is GF(2)-linear with crc(0^k || X) = crc(X) (init 0, no
//    xorout), so a record can be cut into aligned 16-byte "pieces", each
//    piece's contribution computed independently and XORed, provided each is
//    shifted by the number of bytes that follow it.
//  * Work is balanced by bytes: an exclusive scan over per-record "units"
//    (pieces + a fixed per-record charge) gives every wave of a persistent
//    grid an equal slice of the unit space.  A wave walks the records of its
//    slice; records cut by a slice edge are finished by atomic XOR of the
//    partial contributions (XOR is the field addition, so the result does not
//    depend on the order).
//  * Inside a record segment the wave reads 1 KiB per step, fully coalesced
//    (lane l <- bytes [16l, 16l+16) of the step), steps counted backwards
//    from the segment end so the last piece always lands on lane 63.  Each
//    lane keeps a 32-bit register A (Horner over its own pieces, 1 KiB apart).
//    K = 4 steps form a superstep: slot i's tables already include the shift
//    over the (K-1-i) KiB that follow it, so the register is advanced once per
//    superstep.  At the end, lane l's register is shifted by 16*(63-l) bytes
//    (lane-specific tables) and the wave XOR-reduces.
//  * Every table maps a 5-bit slice to a 32-bit contribution.  32 dwords fill
//    the 32 banks of a ds_read_b32 lane group exactly, so every lookup
//    wave-instruction is bank-conflict free whatever the data; the
//    lane-specific tables are laid out [slice][value][lane] so lane l always
//    hits bank l.  No MFMA: this is a byte reduction.
//  * Pieces are read at 16-byte-aligned addresses; bytes outside the record
//    are zeroed (leading zeros are free, trailing z bytes are removed with
//    one inverse shift x^(-8z) on the scalar unit).

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <vector>

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "crc32c_gf2.h"
#include "zdb_crc32.h"
#include "zdb_datafile.h"

namespace {

constexpr int K = ZDBCRC_K;
constexpr int PCH = ZDBCRC_PCH;
constexpr int SCH = ZDBCRC_SCH;
constexpr int WG_PER_CU = 2;              // 2 x 70 KiB of LDS tables per CU
// planning charge per record, in pieces: what a record boundary costs a wave
// (segment reduction, pad shift, metadata, a partly used superstep) measured
// in streaming time -- 384 balances C3 best (16: 0.811 ms, 256: 0.769,
// 384: 0.765, 512: 0.779; profiles/r1/ab_unit_ovh.jsonl)
constexpr uint32_t UNIT_OVH = 384;
constexpr uint64_t MIN_UNITS_PER_WAVE = 256;
// dword offsets inside the per-stream scratch: [0, 16384) one dummy store
// word per wave, [16384, 131072) diagnostic stamps, [131072, 132096) per-CU
// arrival counters (PRIO >= 2), [132096, 136192) tail-pool chunk counters
// (DYN: 2 launch parities x up to 64 pools, one 128-byte line each)
constexpr uint32_t SCRATCH_CU_CTR = 131072;
constexpr uint32_t SCRATCH_DYN_CTR = 132096;
// C5 latency path: small host batches leave their results in a mapped
// host-coherent mailbox: [0] the batch's sequence number, [MAILBOX_PAD ..)
// at most MAILBOX_RECORDS results (publish_kernel)
constexpr uint32_t MAILBOX_PAD = 16;
constexpr uint32_t MAILBOX_RECORDS = 1024;
constexpr uint32_t DYN_MAX_POOLS = 64;
// the tail pool is used only when every slice holds at least this many units
// (so every wave reaches the pool, and every pool has waves to drain it)
constexpr uint64_t DYN_MIN_UNITS_PER_WAVE = 4096;
// ... and no record spans more than this many chunks (each chunk cut of a
// record is one same-address atomic XOR: one huge record would serialise them)
constexpr uint64_t DYN_MAX_CHUNKS_PER_RECORD = 64;
// batches whose records are known to be at most this many bytes take the
// packed kernel (crc_packed_kernel, 768 threads, one load buffer): rows of 16
// lanes up to 4 KiB, of 8 up to 2 KiB, of 4 up to 512 B.  Against the main
// kernel's small-record loop shape (round 2's choice for <= 4 KiB): C2
// 0.766 -> 0.709 ms, C2u 0.800 -> 0.780, Zipf <= 4 KiB 3.64 -> 2.06, 2 KiB
// records 0.939 -> 0.705, Zipf <= 512 B 2.54 -> 0.56
// (profiles/r3/ab_packed_single_buffer*.jsonl)
[[maybe_unused]] constexpr uint64_t SMALL_RECORD_MAX = 4096;
[[maybe_unused]] constexpr uint64_t TINY_RECORD_MAX = 4096;
[[maybe_unused]] constexpr uint64_t TINY8_RECORD_MAX = 2048;
[[maybe_unused]] constexpr uint64_t TINY4_RECORD_MAX = 512;
// record-relative grids of records this long load from the dword below the
// record and fold its last bytes in at the end (next_seg_batched): the fold
// waits for one dword load at the record's end, which small records cannot
// pay for (C2u: 4 KiB values behind 26-byte headers, +8 %) and large ones
// recoup many times over (C3: the 1 MiB values, a third of the bytes, -2.7 %;
// profiles/r2/ab_dword_grid*.jsonl)
constexpr uint64_t DWG_MIN_BYTES = 64 * 1024;

static_assert(ZDBCRC_LDS_DW % 4 == 0, "LDS image must be 16-byte granular");
static_assert(ZDBCRC_LDS_DW * 4 * WG_PER_CU <= 160 * 1024, "LDS budget");

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------

__device__ __forceinline__ uint32_t word_of(const uint4 &v, int d) {
    return d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); // a ^ b ^ c in one VALU op
}

__device__ __forceinline__ uint32_t rotr(uint32_t x, int s) { return __builtin_amdgcn_alignbit(x, x, s); }

// (x on mask m) | (y elsewhere): one v_bfi_b32.  Inline asm so the
// demanded-bits combiner cannot split it into and/and/or.
template <uint32_t M>
__device__ __forceinline__ uint32_t sel(uint32_t x, uint32_t y) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(M), "v"(x), "v"(y));
    return r;
}

// dword byte address of the window in byte n of x: bits [8n+2, 8n+7) of x,
// already scaled by 4 -- one VALU op (v_and_b32, SDWA byte select for n > 0)
// (the compiler finds the SDWA form for bytes 2 and 3 by itself; byte 1 is
// spelled out, it would otherwise emit a shift + and)
__device__ __forceinline__ uint32_t win(uint32_t x, int n) {
    if (n == 0)
        return x & 0x7Cu;
    if (n == 1) {
        uint32_t r;
        asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
            : "=v"(r)
            : "v"(x), "s"(0x7Cu));
        return r;
    }
    return (x >> (8 * n)) & 0x7Cu;
}

// table entry at byte address a of window j's 32-entry table
__device__ __forceinline__ uint32_t look(const uint32_t *tab, int j, uint32_t a) {
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(tab) + j * 128 + a);
}

// contribution of one piece in slot I of a superstep: 26 conflict-free
// lookups over the windows of crc32c_gf2.h (zdbcrc_window_bit), 37 VALU ops
// of index extraction (16 A windows at one op each, two B words at three ops
// + one per window, the C word at five + one per window), folded three at a
// time (v_bitop3 xor3)
// XM (A/B only): 0 = the windows above; 1 = timing diagnostic with one-op
// extraction for every window (wrong checksums)
// TOFF: dword offset of the slot tables in LDS (T; the packed kernel's TP)
template <int I, int XM = 0, uint32_t TOFF = ZDBCRC_OFF_T>
__device__ __forceinline__ uint32_t piece_contrib(const uint4 &v, const uint32_t *lds) {
    const uint32_t *tab = lds + TOFF + I * PCH * 32;
    const uint32_t w0 = v.x, w1 = v.y, w2 = v.z, w3 = v.w;
    if (XM == 3) { // timing diagnostic: the 16 A windows only (wrong checksums)
        uint32_t r = xor3(look(tab, 0, win(w0, 0)), look(tab, 1, win(w0, 1)), look(tab, 2, win(w0, 2)));
        r = xor3(r, look(tab, 3, win(w0, 3)), look(tab, 4, win(w1, 0)));
        r = xor3(r, look(tab, 5, win(w1, 1)), look(tab, 6, win(w1, 2)));
        r = xor3(r, look(tab, 7, win(w1, 3)), look(tab, 8, win(w2, 0)));
        r = xor3(r, look(tab, 9, win(w2, 1)), look(tab, 10, win(w2, 2)));
        r = xor3(r, look(tab, 11, win(w2, 3)), look(tab, 12, win(w3, 0)));
        r = xor3(r, look(tab, 13, win(w3, 1)), look(tab, 14, win(w3, 2)));
        return r ^ look(tab, 15, win(w3, 3));
    }
    if (XM == 1) { // timing diagnostic: 1-op extraction for all 26 (wrong checksums, same LDS pattern)
        uint32_t r = 0;
#pragma unroll
        for (int c = 0; c < PCH; c += 2)
            r = xor3(r, look(tab, c, win(word_of(v, (c >> 2) & 3), c & 3)),
                     look(tab, c + 1, win(word_of(v, ((c + 1) >> 2) & 3), (c + 1) & 3)));
        return r;
    }
    // A: windows 0..15
    uint32_t r = xor3(look(tab, 0, win(w0, 0)), look(tab, 1, win(w0, 1)), look(tab, 2, win(w0, 2)));
    r = xor3(r, look(tab, 3, win(w0, 3)), look(tab, 4, win(w1, 0)));
    r = xor3(r, look(tab, 5, win(w1, 1)), look(tab, 6, win(w1, 2)));
    r = xor3(r, look(tab, 7, win(w1, 3)), look(tab, 8, win(w2, 0)));
    r = xor3(r, look(tab, 9, win(w2, 1)), look(tab, 10, win(w2, 2)));
    r = xor3(r, look(tab, 11, win(w2, 3)), look(tab, 12, win(w3, 0)));
    r = xor3(r, look(tab, 13, win(w3, 1)), look(tab, 14, win(w3, 2)));
    // B: windows 16..23
    const uint32_t u1 = sel<0x1C1C1C1Cu>(rotr(w0, 29), rotr(w1, 27));
    const uint32_t u2 = sel<0x1C1C1C1Cu>(rotr(w2, 29), rotr(w3, 27));
    r = xor3(r, look(tab, 15, win(w3, 3)), look(tab, 16, win(u1, 0)));
    r = xor3(r, look(tab, 17, win(u1, 1)), look(tab, 18, win(u1, 2)));
    r = xor3(r, look(tab, 19, win(u1, 3)), look(tab, 20, win(u2, 0)));
    r = xor3(r, look(tab, 21, win(u2, 1)), look(tab, 22, win(u2, 2)));
    // C: windows 24, 25 (4 index bits each)
    const uint32_t z = sel<0x04040404u>(w1 >> 5, w3 >> 4);
    const uint32_t z2 = sel<0x00300030u>(rotr(z, 6), z);
    r = xor3(r, look(tab, 23, win(u2, 3)), look(tab, 24, z2 & 0x3Cu));
    r ^= look(tab, 25, (z2 >> 16) & 0x3Cu);
    return r;
}

// register advanced over one superstep (tables at dword WOFF: W, K KiB; the
// packed kernel's WP, 1 KiB)
template <uint32_t WOFF>
__device__ __forceinline__ uint32_t advance_superstep_at(uint32_t a, const uint32_t *lds) {
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < SCH; c++)
        r ^= lds[WOFF + c * 32 + ((a >> (5 * c)) & 31u)];
    return r;
}
__device__ __forceinline__ uint32_t advance_superstep(uint32_t a, const uint32_t *lds) {
    return advance_superstep_at<ZDBCRC_OFF_W>(a, lds);
}

// lane l's register shifted by 16*(63-l) bytes; [c][v][lane] layout: bank = lane
__device__ __forceinline__ uint32_t lane_place(uint32_t a, uint32_t lane, const uint32_t *lds) {
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < SCH; c++)
        r ^= lds[ZDBCRC_OFF_L + (c * 32 + ((a >> (5 * c)) & 31u)) * 64 + lane];
    return r;
}

// wave-uniform shift through a global [SCH][32] table (scalar loads)
__device__ __forceinline__ uint32_t uniform_shift(uint32_t x, const uint32_t *__restrict__ tab) {
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < SCH; c++)
        r ^= tab[c * 32 + ((x >> (5 * c)) & 31u)];
    return r;
}

#ifdef ZDBCRC_DIAG
__device__ __forceinline__ uint32_t wave_xor(uint32_t x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
        x ^= __shfl_xor(x, o, 64);
    return x;
}
#endif

// keep bytes [lo, hi) of dword k of a 16-byte piece (0 <= lo <= hi <= 16)
__device__ __forceinline__ uint32_t keep_mask(int lo, int hi, int k) {
    const int a = lo - 4 * k, b = hi - 4 * k;
    const uint32_t mh = b >= 4 ? 0xFFFFFFFFu : b <= 0 ? 0u : ((1u << (8 * b)) - 1u);
    const uint32_t ml = a <= 0 ? 0xFFFFFFFFu : a >= 4 ? 0u : (0xFFFFFFFFu << (8 * a));
    return mh & ml;
}

__device__ __forceinline__ uint4 mask_piece(uint4 v, int lo, int hi) {
    v.x &= keep_mask(lo, hi, 0);
    v.y &= keep_mask(lo, hi, 1);
    v.z &= keep_mask(lo, hi, 2);
    v.w &= keep_mask(lo, hi, 3);
    return v;
}

// Pieces of a record of L > 0 bytes at address a.  Normally the 16-byte
// grid of the address space (aligned loads, first/last piece partial).  When
// that grid costs the record one more 1 KiB step than a grid starting at the
// record itself would (a 4 KiB value after a 26-byte datafile header: 257
// aligned pieces = 5 steps, 256 record-relative pieces = 4), the record uses
// the record-relative grid instead: its loads are byte-misaligned (≈ 20 %
// slower to stream, measured) but it saves a fifth of its lookups.  Only for
// L % 16 == 0, so the last piece ends exactly at the record's end and no load
// leaves the 16-byte blocks the aligned grid reads anyway.  The planner and
// the walk both derive the grid from the piece count.
__host__ __device__ __forceinline__ uint64_t pieces_aligned(uint64_t a, uint64_t L) {
    return ((a + L - 1) >> 4) - (a >> 4) + 1;
}
__host__ __device__ __forceinline__ uint64_t record_pieces(uint64_t a, uint64_t L) {
    const uint64_t na = pieces_aligned(a, L), nr = L >> 4;
    return (L & 15) == 0 && ((nr + 63) >> 6) < ((na + 63) >> 6) ? nr : na;
}

struct SegCtx {
    uint64_t P0;      // 16-aligned address of the record's first piece
    int64_t base_j;   // piece index of (step 0, lane 0); piece = base_j + 64 t + lane
    uint32_t pa;      // first piece of the segment (record-relative)
    uint32_t np;      // pieces in the record
    int lo0;          // first record byte inside piece 0
    int hi_last;      // one past the last record byte inside piece np-1
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 global_u32x4;

// a dword from global memory through a global (not flat) load: a flat load
// counts against lgkmcnt as well as vmcnt and may complete out of order with
// the vector loads, so while one is pending the compiler's waits on LDS
// lookups and payload loads both become full drains
__device__ __forceinline__ uint32_t ld_global_u32(uint64_t a) {
    return *reinterpret_cast<const __attribute__((address_space(1))) uint32_t *>(a);
}

// zero the bytes of a piece that lie outside the record (first/last piece
// only) and whole pieces before the segment (lanes whose load was clamped)
__device__ __forceinline__ uint4 fix_edges(const SegCtx &s, uint4 v, uint32_t t, uint32_t lane) {
    const int64_t jj = s.base_j + 64 * (int64_t)t + (int64_t)lane;
    const bool first = jj == 0, last = jj == (int64_t)s.np - 1;
    if (first || last)
        v = mask_piece(v, first ? s.lo0 : 0, last ? s.hi_last : 16);
    if (jj < (int64_t)s.pa)
        v = make_uint4(0, 0, 0, 0);
    return v;
}

// fix_edges only where the step (64 pieces, wave-uniform range) holds a
// partial first/last piece or lanes before the segment
__device__ __forceinline__ uint4 edge_piece(const SegCtx &s, uint4 v, uint32_t t, uint32_t lane) {
    const int64_t j0 = s.base_j + 64 * (int64_t)t;
    const int64_t jl = (int64_t)s.np - 1;
    const bool need = j0 < (int64_t)s.pa || (s.lo0 != 0 && j0 <= 0 && 0 <= j0 + 63) ||
                      (s.hi_last != 16 && j0 <= jl && jl <= j0 + 63);
    return need ? fix_edges(s, v, t, lane) : v;
}

// one superstep (K steps) folded into the lane register.  Only the first
// superstep can hold empty leading steps / lanes and the record's first
// piece; only the last can hold the record's last piece: EDGE enables the
// checks there, the middle supersteps run without them.
template <bool EDGE, int XM = 0>
__device__ __forceinline__ uint32_t superstep(const SegCtx &s, uint32_t acc, const uint4 (&cur)[K], uint32_t ss,
                                              uint32_t t0, uint32_t lane, const uint32_t *lds) {
    if (ss)
        acc = advance_superstep(acc, lds);
    const uint32_t tb = ss * K;
#define ZDBCRC_SLOT(I)                                                                   \
    if (!EDGE || tb + I >= t0)                                                           \
        acc ^= piece_contrib<I, XM>(EDGE ? edge_piece(s, cur[I], tb + I, lane) : cur[I], lds);

    ZDBCRC_SLOT(0)
    ZDBCRC_SLOT(1)
    ZDBCRC_SLOT(2)
    ZDBCRC_SLOT(3)
#undef ZDBCRC_SLOT
    return acc;
}

static_assert(K == 4, "superstep unrolls 4 slots");

// A record segment as the wave walks it (all fields wave-uniform).
struct Seg {
    SegCtx c;
    uint64_t us;   // unit index of the record's first piece
    uint64_t r;    // record index
    uint32_t pb;   // one past the segment's last piece (record-relative)
    uint32_t S;    // supersteps in the segment
    uint32_t t0;   // first non-empty step
    uint32_t z;    // zero bytes padding the record's last piece
};

// ---------------------------------------------------------------------------
// v3: pipelined stream + lane-parallel record metadata + DPP reduction
// ---------------------------------------------------------------------------

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// XOR of a value over the 64 lanes, as a wave-uniform scalar: DPP within
// rows of 16 (VALU, no LDS traffic), then four readlanes
__device__ __forceinline__ uint32_t wave_xor_scalar(uint32_t x) {
    x ^= __builtin_amdgcn_update_dpp(0u, x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    x ^= __builtin_amdgcn_update_dpp(0u, x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    x ^= __builtin_amdgcn_update_dpp(0u, x, 0x124, 0xF, 0xF, false); // row_ror:4
    x ^= __builtin_amdgcn_update_dpp(0u, x, 0x128, 0xF, 0xF, false); // row_ror:8
    return __builtin_amdgcn_readlane(x, 0) ^ __builtin_amdgcn_readlane(x, 16) ^
           __builtin_amdgcn_readlane(x, 32) ^ __builtin_amdgcn_readlane(x, 48);
}

// per-record unit prefix as the planner leaves it: local[r] is the prefix
// inside r's block of 2^lg records and boff[b] (built in LDS by every
// workgroup from the planner's block totals) the prefix of whole blocks:
// unit_start(r) = local[r] + boff[r >> lg].  boff == nullptr when local
// already holds the global prefix (host-planned batches).
constexpr uint32_t PLAN_MAX_BLOCKS = 1024; // block offsets kept in LDS
struct UnitPrefix {
    const uint64_t *local;
    const uint64_t *boff;
    uint32_t lg;
    __device__ __forceinline__ uint64_t operator()(uint64_t r) const {
        return boff ? local[r] + boff[r >> lg] : local[r];
    }
};

// what the planner hands the checksum kernel
struct PlanArgs {
    const uint64_t *local; // n + 1 entries
    const uint64_t *bsum;  // nb block totals (nullptr: local is global)
    uint32_t nb;
    uint32_t lg;
    const uint32_t *bmax; // nb block maxima of a record's unit count (tail-pool guard)
    const uint64_t *dn;   // nullptr, or the record count in device memory (n is then its bound)
    uint32_t cls_max;     // packed kernel of a split batch: only records of at most this many bytes are its
                          // (the others -- no units in its plan -- belong to the main kernel); 0: all
};

__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t y = (uint32_t)__shfl_xor((int)x, o, 64);
        x = y > x ? y : x;
    }
    return x;
}

// record r with unit_start[r] <= b < unit_start[r+1]: 64-way search, one
// vector load per round (3 rounds for 1e5 records, 4 for 1e6)
__device__ __forceinline__ uint64_t find_record(const UnitPrefix &unit_start, uint64_t n, uint64_t b,
                                                uint32_t lane) {
    uint64_t lo = 0, hi = n;
    while (hi - lo > 1) {
        const uint64_t step = (hi - lo + 63) >> 6;
        const uint64_t idx = lo + (uint64_t)lane * step;
        const bool le = idx < hi && unit_start(idx) <= b;
        const uint64_t mask = __ballot(le);
        const uint32_t L = 63u - (uint32_t)__clzll(mask);
        lo += (uint64_t)L * step;
        const uint64_t h2 = lo + step;
        hi = h2 < hi ? h2 : hi;
    }
    return lo;
}

// the same search through the planner's block structure: the block from the
// offsets in LDS (two LDS rounds), then the block's records in ONE round of
// global loads (up to 4 per lane, issued together; the prefix is monotone,
// so the answer is the count of records at or below b) -- one HBM round trip
// instead of one per 64-way round (3 for C3's 86,959 records, 4 for 1 M)
__device__ __forceinline__ uint64_t find_record_blocked(const UnitPrefix &unit_start, uint32_t nb, uint64_t n,
                                                        uint64_t b, uint32_t lane) {
    if (!unit_start.boff || nb == 0)
        return find_record(unit_start, n, b, lane);
    uint64_t lo = 0, hi = nb; // last block bi with boff[bi] <= b
    while (hi - lo > 1) {
        const uint64_t step = (hi - lo + 63) >> 6;
        const uint64_t idx = lo + (uint64_t)lane * step;
        const uint64_t mask = __ballot(idx < hi && unit_start.boff[idx] <= b);
        const uint32_t L = 63u - (uint32_t)__clzll(mask);
        lo += (uint64_t)L * step;
        const uint64_t h2 = lo + step;
        hi = h2 < hi ? h2 : hi;
    }
    const uint64_t bo = unit_start.boff[lo];
    const uint64_t r0 = lo << unit_start.lg;
    const uint64_t r1 = ((lo + 1) << unit_start.lg) < n ? ((lo + 1) << unit_start.lg) : n;
    const uint64_t q = (r1 - r0 + 63) >> 6;
    if (q > 4) { // blocks of more than 256 records: 64-way rounds inside the block
        uint64_t a = r0, z = r1;
        while (z - a > 1) {
            const uint64_t step = (z - a + 63) >> 6;
            const uint64_t idx = a + (uint64_t)lane * step;
            const uint64_t mask = __ballot(idx < z && unit_start.local[idx] + bo <= b);
            const uint32_t L = 63u - (uint32_t)__clzll(mask);
            a += (uint64_t)L * step;
            const uint64_t h2 = a + step;
            z = h2 < z ? h2 : z;
        }
        return a;
    }
    uint64_t v[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
        const uint64_t idx = r0 + 64u * k + lane;
        v[k] = k < q && idx < r1 ? unit_start.local[idx] : ~0ull;
    }
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++)
        cnt += (uint32_t)__popcll(__ballot(v[k] != ~0ull && v[k] + bo <= b));
    return r0 + cnt - 1;
}

// metadata of 64 consecutive records [rb, rb+64), record rb+l on lane l
struct MetaBatch {
    uint64_t rb;   // uniform
    uint64_t u0;   // unit_start[r]
    uint64_t ur;   // unit_start[r+1]
    uint64_t addr; // arena address of the record
    uint32_t len;
};

__device__ __forceinline__ void load_meta(MetaBatch &m, uint64_t rb, uint64_t n, uint32_t lane,
                                          const UnitPrefix &unit_start, const uint8_t *arena,
                                          const uint64_t *__restrict__ offsets,
                                          const uint32_t *__restrict__ lengths) {
    m.rb = rb;
    const uint64_t r = rb + lane;
    m.u0 = ~0ull;
    m.ur = ~0ull;
    m.addr = 0;
    m.len = 0;
    if (r < n) {
        m.u0 = unit_start(r);
        m.ur = unit_start(r + 1);
        m.addr = reinterpret_cast<uint64_t>(arena) + offsets[r];
        m.len = lengths[r];
    }
}

template <uint32_t UO, bool BMG = false, uint64_t DWGM = DWG_MIN_BYTES>
__device__ __forceinline__ bool next_seg_batched(uint64_t &r, uint64_t n, uint64_t ub, uint64_t ue, uint32_t lane,
                                                 MetaBatch &m, const UnitPrefix &unit_start,
                                                 const uint8_t *arena, const uint64_t *__restrict__ offsets,
                                                 const uint32_t *__restrict__ lengths, Seg &sg) {
    for (;;) {
        if (r >= n)
            return false;
        if (r >= m.rb + 64)
            load_meta(m, r, n, lane, unit_start, arena, offsets, lengths);
        const uint32_t li = (uint32_t)(r - m.rb);
        const uint64_t u0 = readlane64(m.u0, li);
        if (u0 >= ue)
            return false;
        const uint64_t us = u0 + UO;
        const uint64_t ur = readlane64(m.ur, li);
        const uint64_t s_lo = ub > us ? ub : us;
        const uint64_t s_hi = ue < ur ? ue : ur;
        if (s_hi > s_lo) {
            const uint64_t A = readlane64(m.addr, li);
            // (the builtin returns int: a length of 2 GiB or more must not be sign-extended)
            const uint64_t Aend = A + (uint32_t)__builtin_amdgcn_readlane(m.len, li);
            sg.r = r;
            sg.us = us;
            sg.c.np = (uint32_t)(ur - us);
            // record-relative grid iff the planner counted fewer pieces than
            // the aligned grid has (record_pieces).  For records of at least
            // DWG_MIN_BYTES its loads start at the dword below the record
            // (byte-misaligned 16-byte loads stream ~20 % slower than
            // dword-aligned ones, misalign_probe.jsonl): the h = A mod 4 bytes
            // before the record are masked off and the record's last h bytes,
            // which the grid then misses, are folded in at its end
            // (seg_value_v3, z = 16 + h); aligned grid: z = the trailing pad of
            // the last piece.  BMG (A/B only): byte-misaligned loads for all
            const bool rel = sg.c.np != (uint32_t)pieces_aligned(A, Aend - A);
            const uint32_t h = rel && !BMG && Aend - A >= DWGM ? (uint32_t)(A & 3u) : 0u;
            sg.c.P0 = rel ? A - h : (A & ~15ull);
            sg.z = rel ? (h ? 16u + h : 0u) : (uint32_t)(sg.c.P0 + 16u * (uint64_t)sg.c.np - Aend);
            sg.c.lo0 = rel ? (int)h : (int)(A & 15u);
            sg.c.hi_last = rel ? 16 : 16 - (int)sg.z;
            sg.c.pa = (uint32_t)(s_lo - us);
            sg.pb = (uint32_t)(s_hi - us);
            const uint32_t T = (sg.pb - sg.c.pa + 63u) / 64u;
            sg.S = (T + K - 1) / K;
            sg.t0 = sg.S * K - T;
            sg.c.base_j = (int64_t)sg.pb - 64 * (int64_t)sg.S * K;
            r++;
            return true;
        }
        r++;
    }
}

// loads of superstep ss: uniform base (segment's first piece) + 32-bit lane
// offset; lanes before the segment re-read its first piece (zeroed later)
// TEL (with NTL): as pk_load's -- the lanes reaching the line of the
// superstep's last byte load without the nontemporal hint
template <bool NTL = false, bool NOLOAD = false, int TEL = 0>
__device__ __forceinline__ void load_superstep_v3(const SegCtx &s, uint32_t ss, uint32_t lane, uint4 (&buf)[K]) {
    const uint64_t base = s.P0 + 16u * (uint64_t)s.pa;
    const int32_t rel0 = (int32_t)(s.base_j - (int64_t)s.pa) + 64 * (int32_t)(ss * K) + (int32_t)lane;
#pragma unroll
    for (int i = 0; i < K; i++) {
        int32_t rel = rel0 + 64 * i;
        rel = rel < 0 ? 0 : rel;
        global_u32x4 *p = reinterpret_cast<global_u32x4 *>(base + ((uint64_t)(uint32_t)rel << 4));
        if (NOLOAD) { // timing diagnostic: no memory traffic, data made up from the address
            const uint32_t a = (uint32_t)reinterpret_cast<uint64_t>(p);
            buf[i] = make_uint4(a, a * 0x9E3779B9u, a ^ 0x5bd1e995u, a + ss);
            continue;
        }
        u32x4 v;
        if constexpr (NTL && TEL > 0) {
            const uint64_t a = reinterpret_cast<uint64_t>(p);
            const uint64_t last = base + ((uint64_t)(uint32_t)(rel0 - (int32_t)lane + 64 * K - 1) << 4) + 15;
            if (i == K - 1 && ((a + 15) >> 7) == (last >> 7))
                v = *p;
            else
                v = __builtin_nontemporal_load(p);
        } else {
            v = NTL ? __builtin_nontemporal_load(p) : *p;
        }
        buf[i] = make_uint4(v.x, v.y, v.z, v.w);
    }
}

template <int NOZ = 0>
__device__ __forceinline__ uint32_t seg_value_v3(const Seg &sg, uint32_t acc, uint32_t lane, const uint32_t *lds,
                                                 const uint32_t *__restrict__ tables) {
    // record-relative grid from the dword below the record (z = 16 + h): the
    // segment that ends the record folds in its last h bytes y (one aligned
    // dword, loaded before the reduction so that its latency hides behind it),
    // crc(X || y) = shift(crc(X) ^ y, h); the other segments only shift by h
    const bool fold = sg.z >= 16u;
    uint32_t y = 0;
    if (fold && sg.pb == sg.c.np)
        y = ld_global_u32(sg.c.P0 + 16u * (uint64_t)sg.c.np) & ((1u << (8u * (sg.z - 16u))) - 1u);
    uint32_t x = wave_xor_scalar(NOZ >= 2 ? acc : lane_place(acc, lane, lds));
    if (fold)
        x = uniform_shift(x ^ y, tables + ZDBCRC_OFF_F + (sg.z - 16u) * SCH * 32);
    else if (!NOZ && sg.z)
        x = uniform_shift(x, tables + ZDBCRC_OFF_Z + sg.z * SCH * 32);
    // shift over the record pieces after the segment: one round per nonzero
    // radix-256 digit (at most 4 dependent table reads, usually 0-2)
    uint32_t q = sg.c.np - sg.pb;
    for (int j = 0; q; j++, q >>= 8)
        if (q & 255u)
            x = uniform_shift(x, tables + ZDBCRC_OFF_R + (j * 256 + (q & 255u)) * SCH * 32);
    return x;
}

__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v, uint32_t lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t t = __shfl_up(v, o, 64);
        if (lane >= (uint32_t)o)
            v += t;
    }
    return v;
}

// exclusive scan of one value per thread across an NT-thread block;
// *total = the sum; wsum: 2 (NT / 64) + 1 entries of LDS
template <uint32_t NT>
__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t v, uint64_t *wsum, uint64_t *total) {
    constexpr uint32_t NW = NT / 64;
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    const uint64_t incl = wave_incl_scan64(v, lane);
    if (lane == 63)
        wsum[wid] = incl;
    __syncthreads();
    if (wid == 0) {
        const uint64_t w = lane < NW ? wsum[lane] : 0;
        const uint64_t wi = wave_incl_scan64(w, lane);
        if (lane < NW)
            wsum[NW + lane] = wi - w;
        if (lane == NW - 1)
            wsum[2 * NW] = wi;
    }
    __syncthreads();
    *total = wsum[2 * NW];
    const uint64_t r = incl - v + wsum[NW + wid];
    __syncthreads(); // wsum reusable
    return r;
}

// STAMP (diagnostic build only): each wave writes its start/end
// s_memrealtime to scratch[16384 + 4 gw ...] -- never read by the kernel
// PRIO: waves of a workgroup publish their progress in LDS every other
// superstep and the slower half raises its issue priority (s_setprio 3).
// Without it the co-resident waves of a CU finish up to 2x apart (age-ordered
// arbitration; measured with the STAMP build) and the kernel ends on a tail.
// PRIO 2/3: the same, plus the two workgroups sharing a CU are told apart
// (arrival order at a per-CU counter, keyed by the hardware CU id): issue
// arbitration favours the older workgroup, so the younger one runs on a
// priority one step (2) or two steps (3) above it.
// NOZ: timing diagnostic only (1: skips the trailing-pad shift, 2: also the
// lane placement -- wrong checksums)
// NTL: payload loads carry the nontemporal hint (read once, never reused)
// NOLOAD: timing diagnostic only (no payload loads: the compute floor; wrong checksums)
// PP: the loop is unrolled twice and the two load buffers swap roles instead
// of being copied (16 v_mov per superstep); 1 = always, 2 = only when every
// record of the batch fits one superstep (planner block maxima), 3 = always,
// waiting for the previous loads before issuing the next (one superstep of
// loads in flight per wave, as the copying loop has)
// DYN > 0: tail pool.  Static slices cover the first (16 - DYN)/16 of the unit
// space; the rest is split into DYN_POOLS pools (pool = blockIdx mod DYN_POOLS) of
// CPW chunks per wave, claimed with one atomicAdd each as waves run out of
// work, so waves that the arbitration favours take more of the tail and the
// launch does not end on its slowest waves.  Cut partials of finished ranges
// are flushed with atomic XOR at each claim (at most 2 are pending then).
template <int WGT, int WPE, bool STAMP = false, int PRIO = 0, uint32_t UO = UNIT_OVH, int NOZ = 0,
          bool NTL = false, bool NOLOAD = false, int XM = 0, int DYN = 0, int CPW = 4, uint32_t DYN_POOLS = 8,
          bool SP = false, int PP = 0, bool SEGDUMP = false, bool BMG = false, bool XP = false,
          uint64_t DWGM = DWG_MIN_BYTES, bool FRB = false, bool SB1 = false, int TEL = 0>
__global__ __launch_bounds__(WGT, WPE) void crc_batch_kernel_v3(
    const uint8_t *__restrict__ arena, const uint64_t *__restrict__ offsets,
    const uint32_t *__restrict__ lengths, const PlanArgs plan, uint64_t n,
    uint32_t *__restrict__ out, const uint32_t *__restrict__ tables, uint32_t max_waves,
    uint32_t *__restrict__ scratch, uint32_t epoch) {
    constexpr uint32_t NW = WGT / 64, NSLOT = 2 * NW;
    if (plan.dn) { // the record count left in device memory by the producer (f3 walk): n is its bound
        const uint64_t dn = *plan.dn;
        n = dn < n ? dn : n;
    }
    __shared__ __attribute__((aligned(16))) uint32_t lds[ZDBCRC_LDS_DW + 16 + 2 * NSLOT];
    __shared__ uint64_t boff[PLAN_MAX_BLOCKS + 1];
    __shared__ uint64_t wsum[2 * NW + 1];
    __shared__ uint32_t wmax[NW];
    uint32_t *const prog = lds + ZDBCRC_LDS_DW;   // per-wave progress (PRIO)
    uint32_t *const slot = prog + 16;             // cut records of the workgroup: [NSLOT] r, [NSLOT] x
    const uint64_t t_start = STAMP ? __builtin_amdgcn_s_memrealtime() : 0;

    // block offsets of the unit prefix (planner block totals, scanned here)
    UnitPrefix unit_start{plan.local, nullptr, plan.lg};
    if (plan.bsum) {
        constexpr uint32_t PER = (PLAN_MAX_BLOCKS + WGT - 1) / WGT;
        uint64_t v[PER], t = 0;
        uint32_t mx = 0;
#pragma unroll
        for (uint32_t i = 0; i < PER; i++) {
            const uint32_t b = threadIdx.x * PER + i;
            v[i] = b < plan.nb ? plan.bsum[b] : 0;
            t += v[i];
            if (DYN || PP == 2) {
                const uint32_t q = b < plan.nb ? plan.bmax[b] : 0u;
                mx = q > mx ? q : mx;
            }
        }
        if (DYN || PP == 2) {
            mx = wave_max(mx);
            if ((threadIdx.x & 63u) == 0)
                wmax[threadIdx.x >> 6] = mx;
        }
        uint64_t total;
        uint64_t e = block_excl_scan64<WGT>(t, wsum, &total);
#pragma unroll
        for (uint32_t i = 0; i < PER; i++) {
            const uint32_t b = threadIdx.x * PER + i;
            if (b <= plan.nb)
                boff[b] = e;
            e += v[i];
        }
        __syncthreads();
        unit_start.boff = boff;
    }

    // locate this wave's slice and issue its first loads before the table
    // fill, so the first HBM round trip overlaps the LDS copy; every wave
    // reaches the barrier below, active or not
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gw = __builtin_amdgcn_readfirstlane(blockIdx.x * (WGT / 64) + (threadIdx.x >> 6));
    const uint64_t total = unit_start(n);
    uint64_t nwaves = (total + MIN_UNITS_PER_WAVE - 1) / MIN_UNITS_PER_WAVE;
    if (nwaves > max_waves)
        nwaves = max_waves;
    // tail pool only with a full grid whose slices are all long enough
    bool dyn = DYN > 0 && plan.bmax && gridDim.x >= DYN_POOLS && total >= DYN_MIN_UNITS_PER_WAVE * max_waves;
    if (dyn) { // largest record vs chunk size (wmax written before the scan's barriers)
        uint32_t mxu = 0;
        for (uint32_t i = 0; i < NW; i++)
            mxu = wmax[i] > mxu ? wmax[i] : mxu;
        const uint64_t chunk = total * DYN / 16 / ((uint64_t)CPW * nwaves);
        dyn = mxu <= DYN_MAX_CHUNKS_PER_RECORD * chunk;
    }
    bool pp = PP == 1 || PP == 3;
    if (PP == 2 && plan.bmax) { // every record within one superstep (+1 piece of misalignment)
        uint32_t mxu = 0;
        for (uint32_t i = 0; i < NW; i++)
            mxu = wmax[i] > mxu ? wmax[i] : mxu;
        pp = mxu <= UO + 64u * K + 1u;
    }
    const uint64_t Ts = dyn ? total - total * DYN / 16 : total;
    uint64_t ub = Ts * gw / nwaves;
    uint64_t ue = Ts * (gw + 1) / nwaves;
    bool active = gw < nwaves && ub < ue;
    MetaBatch m;
    m.rb = ~0ull;
    uint64_t rn = 0;
    Seg cur, nx;
    uint4 bufc[K], bufn[K];
    if (active) {
        rn = FRB ? find_record_blocked(unit_start, plan.nb, n, ub, lane) : find_record(unit_start, n, ub, lane);
        load_meta(m, rn, n, lane, unit_start, arena, offsets, lengths);
        active = next_seg_batched<UO, BMG, DWGM>(rn, n, ub, ue, lane, m, unit_start, arena, offsets, lengths, cur);
        if (active)
            load_superstep_v3<NTL, NOLOAD, TEL>(cur.c, 0, lane, bufc);
    }
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (PRIO && lane == 0)
        prog[wid] = active ? 0u : 0xFFFFFFFFu; // an idle wave counts as ahead of everyone
    if (lane < 2)
        slot[2 * wid + lane] = ~0u;
    if (PRIO >= 2 && threadIdx.x == 0) {
        // arrival order of this workgroup on its CU (parity of a per-CU
        // counter that every launch advances by the CU's workgroup count)
        const uint32_t hw = __builtin_amdgcn_s_getreg(0xF804);  // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg(0xF814); // HW_REG_XCC_ID
        const uint32_t key = ((xcc & 7u) << 7) | (((hw >> 13) & 7u) << 5) | (((hw >> 12) & 1u) << 4) | ((hw >> 8) & 15u);
        prog[15] = atomicAdd(scratch + SCRATCH_CU_CTR + key, 1u) & 1u;
    }
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(tables);
        uint4 *dst = reinterpret_cast<uint4 *>(lds);
        for (int i = threadIdx.x; i < ZDBCRC_LDS_DW / 4; i += WGT)
            dst[i] = src[i];
    }
    if (blockIdx.x == 0 && threadIdx.x < DYN_MAX_POOLS) // the next launch's counters (every variant)
        scratch[SCRATCH_DYN_CTR + (((epoch + 1u) & 1u) * DYN_MAX_POOLS + threadIdx.x) * 32u] = 0u;
    __syncthreads();

    uint64_t cut_r[2] = {0, 0};
    uint32_t cut_x[2] = {0, 0}, ncut = 0;
    uint64_t pbase = 0; // units of earlier ranges (PRIO progress)
    // tail pool of this workgroup: chunk c covers [P0 + PL c / nch, P0 + PL (c+1) / nch)
    // XP: the workgroups of a pool come from every XCD (workgroup b runs on XCD
    // b mod 8), so that a slower XCD's share of the pool is taken by the
    // others: each run of DYN_POOLS consecutive workgroups covers every pool
    // once (so any grid of >= DYN_POOLS workgroups serves every pool, as the
    // guard above requires), rotated by one per run (pool p gets XCDs p,
    // p - 1, ..., p - 15 mod 8 of a 512-workgroup grid: each twice)
    const uint32_t pool = (XP ? blockIdx.x + blockIdx.x / DYN_POOLS : blockIdx.x) % DYN_POOLS;
    const uint64_t Td = total - Ts;
    const uint64_t P0 = Ts + Td * pool / DYN_POOLS;
    const uint64_t PL = Ts + Td * (pool + 1) / DYN_POOLS - P0;
    const uint64_t nch = (uint64_t)CPW * (nwaves / DYN_POOLS);
    static_assert(DYN_POOLS <= DYN_MAX_POOLS, "tail-pool counters");
    uint32_t *const ctr = scratch + SCRATCH_DYN_CTR + ((epoch & 1u) * DYN_MAX_POOLS + pool) * 32u;
    // next range from the pool; false once the pool is drained
    auto claim = [&](Seg &sg) -> bool {
        if (SP) // SP: waves still in their static slice issue ahead of pool waves
                // (C3 -1 to -2 %, profiles/r1/ab_dyn_sp*.jsonl)
            __builtin_amdgcn_s_setprio(0);
        if (lane == 0) {
            if (ncut > 0)
                atomicXor(out + cut_r[0], cut_x[0]);
            if (ncut > 1)
                atomicXor(out + cut_r[1], cut_x[1]);
        }
        ncut = 0;
        for (;;) {
            uint32_t c = 0;
            if (lane == 0)
                c = atomicAdd(ctr, 1u);
            c = __builtin_amdgcn_readfirstlane(c);
            if (c >= nch)
                return false;
            pbase += ue - ub;
            ub = P0 + PL * c / nch;
            ue = P0 + PL * (c + 1) / nch;
            if (ue <= ub)
                continue;
            rn = FRB ? find_record_blocked(unit_start, plan.nb, n, ub, lane) : find_record(unit_start, n, ub, lane);
            if (rn < m.rb)
                load_meta(m, rn, n, lane, unit_start, arena, offsets, lengths);
            if (next_seg_batched<UO, BMG, DWGM>(rn, n, ub, ue, lane, m, unit_start, arena, offsets, lengths, sg))
                return true;
        }
    };
    if (SP && dyn)
        __builtin_amdgcn_s_setprio(2);
    if (!active) {
        if (!(DYN && dyn && claim(cur)))
            return;
        load_superstep_v3<NTL, NOLOAD, TEL>(cur.c, 0, lane, bufc);
    }
    const uint32_t young = PRIO >= 2 ? __builtin_amdgcn_readfirstlane(prog[15]) : 0u;

    uint32_t *const dummy = scratch + gw;
    uint32_t css = 0, acc = 0, iter = 0;
    // one superstep of the current segment (the loads of the next one are
    // issued first); leaves `more` false once the wave's work is done
#define ZDBCRC_STEP(BUFC, BUFN)                                                                               \
        if (PRIO && (++iter & 1) == 0) {                                                                      \
            const uint32_t mine = (uint32_t)(pbase + cur.us + cur.c.pa + 64u * K * css - ub);                 \
            if (lane == 0)                                                                                    \
                prog[wid] = mine;                                                                             \
            const uint32_t other = lane < (uint32_t)(WGT / 64) ? prog[lane] : 0u;                             \
            const uint32_t ahead = (uint32_t)__popcll(__ballot(other > mine));                                \
            const bool slow = ahead >= (uint32_t)(WGT / 128);                                                 \
            if (PRIO == 1) {                                                                                  \
                if (slow)                                                                                     \
                    __builtin_amdgcn_s_setprio(3);                                                            \
                else                                                                                          \
                    __builtin_amdgcn_s_setprio(0);                                                            \
            } else if (PRIO == 2) {                                                                           \
                if (slow) {                                                                                   \
                    if (young)                                                                                \
                        __builtin_amdgcn_s_setprio(3);                                                        \
                    else                                                                                      \
                        __builtin_amdgcn_s_setprio(2);                                                        \
                } else {                                                                                      \
                    if (young)                                                                                \
                        __builtin_amdgcn_s_setprio(1);                                                        \
                    else                                                                                      \
                        __builtin_amdgcn_s_setprio(0);                                                        \
                }                                                                                             \
            } else {                                                                                          \
                if (young) {                                                                                  \
                    if (slow)                                                                                 \
                        __builtin_amdgcn_s_setprio(3);                                                        \
                    else                                                                                      \
                        __builtin_amdgcn_s_setprio(2);                                                        \
                } else {                                                                                      \
                    if (slow)                                                                                 \
                        __builtin_amdgcn_s_setprio(1);                                                        \
                    else                                                                                      \
                        __builtin_amdgcn_s_setprio(0);                                                        \
                }                                                                                             \
            }                                                                                                 \
        }                                                                                                     \
        uint32_t nss = 0;                                                                                     \
        bool more = true;                                                                                     \
        if (css + 1 < cur.S) {                                                                                \
            nx = cur;                                                                                         \
            nss = css + 1;                                                                                    \
        } else if (!next_seg_batched<UO, BMG, DWGM>(rn, n, ub, ue, lane, m, unit_start, arena, offsets, lengths, nx) &&  \
                   !(DYN && dyn && claim(nx))) {                                                              \
            more = false;                                                                                     \
            nx = cur;                                                                                         \
            nss = css;                                                                                        \
        }                                                                                                     \
        if (PP == 3)                                                                                          \
            __builtin_amdgcn_s_waitcnt(0x0F70);                                                               \
        if (!SB1)                                                                                             \
            load_superstep_v3<NTL, NOLOAD, TEL>(nx.c, nss, lane, BUFN);                                            \
        if (css == 0 || css + 1 == cur.S)                                                                     \
            acc = superstep<true, XM>(cur.c, acc, BUFC, css, cur.t0, lane, lds);                              \
        else                                                                                                  \
            acc = superstep<false, XM>(cur.c, acc, BUFC, css, cur.t0, lane, lds);                             \
        uint32_t *dst = dummy;                                                                                \
        uint32_t x = 0;                                                                                       \
        if (css + 1 == cur.S) {                                                                               \
            x = seg_value_v3<NOZ>(cur, acc, lane, lds, tables);                                               \
            if (SEGDUMP && lane == 0) {                                                                       \
                uint64_t *sd = reinterpret_cast<uint64_t *>(scratch + 16384) + 4 * gw;                        \
                sd[0] = cur.c.pa;                                                                             \
                sd[1] = cur.pb;                                                                               \
                sd[2] = x;                                                                                    \
                sd[3] = cur.r | ((uint64_t)cur.c.np << 32);                                                   \
            }                                                                                                 \
            acc = 0;                                                                                          \
            if (cur.c.pa == 0 && cur.pb == cur.c.np) {                                                        \
                dst = out + cur.r;                                                                            \
            } else {                                                                                          \
                cut_r[ncut & 1] = cur.r;                                                                      \
                cut_x[ncut & 1] = x;                                                                          \
                ncut++;                                                                                       \
            }                                                                                                 \
        }                                                                                                     \
        if (lane == 0)                                                                                        \
            *dst = x;                                                                                         \
        if (SB1 && more) /* one load buffer: the next superstep's loads after the fold */                    \
            load_superstep_v3<NTL, NOLOAD, TEL>(nx.c, nss, lane, BUFC);

    if (PP && pp) { // ping-pong: the two load buffers swap roles, no register copies
        for (;;) {
            {
                ZDBCRC_STEP(bufc, bufn)
                if (!more)
                    break;
                cur = nx;
                css = nss;
            }
            {
                ZDBCRC_STEP(bufn, bufc)
                if (!more)
                    break;
                cur = nx;
                css = nss;
            }
        }
    } else {
        for (;;) {
            ZDBCRC_STEP(bufc, bufn)
            if (!more)
                break;
            cur = nx;
            css = nss;
            if (!SB1) {
#pragma unroll
                for (int i = 0; i < K; i++)
                    bufc[i] = bufn[i];
            }
        }
    }
#undef ZDBCRC_STEP
    if (PRIO && lane == 0)
        prog[wid] = 0xFFFFFFFFu; // finished: counts as ahead of everyone
    if (STAMP && lane == 0) {
        uint64_t *st = reinterpret_cast<uint64_t *>(scratch + 16384) + 4 * gw;
        st[0] = t_start;
        st[1] = __builtin_amdgcn_s_memrealtime();
        st[2] = __builtin_amdgcn_s_getreg(0xF804); // HW_REG_HW_ID: wave/simd/cu/se
        st[3] = __builtin_amdgcn_s_getreg(0xF814); // HW_REG_XCC_ID
    }
    // records cut by a slice edge: combine the workgroup's partial values in
    // LDS first (consecutive waves cut the same record; a record spanning many
    // slices would otherwise take one same-address atomic per wave), then one
    // atomic XOR per distinct record.  Waves that left early are not counted
    // by the barrier; their slots hold ~0.
    if (lane < 2 && lane < ncut) {
        slot[2 * wid + lane] = (uint32_t)cut_r[lane];
        slot[NSLOT + 2 * wid + lane] = cut_x[lane];
    }
    __syncthreads();
    const uint32_t r_l = lane < NSLOT ? slot[lane] : ~0u;
    const uint32_t x_l = lane < NSLOT ? slot[NSLOT + lane] : 0u;
#pragma unroll
    for (uint32_t i = 0; i < 2; i++) {
        const uint32_t s_i = 2 * wid + i;
        const uint32_t r_s = __builtin_amdgcn_readlane(r_l, s_i);
        if (r_s == ~0u)
            continue;
        if (__ballot(lane < s_i && r_l == r_s) != 0)
            continue; // a lower slot owns this record
        const uint32_t v = wave_xor_scalar(r_l == r_s ? x_l : 0u);
        if (lane == 0)
            atomicXor(out + r_s, v);
    }
}

// ---------------------------------------------------------------------------
// packed small-record kernel: four records per wave, one per row of 16 lanes
// ---------------------------------------------------------------------------
//
// The main kernel walks one record at a time with the whole wave, so a 4 KiB
// value costs it one superstep plus everything a record boundary costs (lane
// placement, reduction, metadata readlanes, segment bookkeeping: ~60 VALU and
// ~140 SALU per record, the C2/C2u gap to C3; zipf_small in
// profiles/r3/ab_split_small_large.jsonl: 2.96 us of wave time per record of
// <= 4 KiB).  Here row g of a wave (lanes 16g .. 16g+15) walks a record of
// its own: a slot is 256 B of it (16 lanes x 16 B), a superstep 1 KiB, and
// the four rows of a packet share every instruction; a packet takes as many
// supersteps as its longest record.  Placement, DPP reduction, fold and
// store happen once per packet, not once per record.
//
// Grid of a record [A, E): the pieces end at Ep, the dword at or below E, so
// every load is dword-aligned (byte-misaligned 16-byte loads stream ~19 %
// slower, profiles/r2/misalign_probe.jsonl); the h = min(E & 3, L) bytes y
// after Ep are folded in at the end, crc(X || y) = shift(crc(X) ^ y, h).
// Piece 0 starts lo0 = 16 np - (L - h) bytes before A; those bytes are
// masked.  Nothing is read past ceil4(E), and below A only inside piece 0 --
// in A's 4 KiB page unless A lies in the first 16 bytes of a page: then piece
// 0 is loaded from A's aligned block and moved up in registers (`d`, rare).
//
// Position q = 64 s + 16 i + l16 of a row's packet stream (superstep s, slot
// i, lane l16) holds piece k = q - kb, kb = 64 S - np (k < 0: empty), loaded
// from Ep - 16 (64 S - q).  Its contribution is shifted by 16 (64 S - 1 - q)
// bytes: TP[i] carries 256 (3 - i), WP advances 1 KiB per superstep and LP
// places lane l16 by 16 (15 - l16).  CPU model: tests/kernel_model.py
// packed_batch.
//
// Work split: the planner's unit prefix (pieces + UO_PK per record); a wave
// owns the records whose first unit lies in its slice (records are never
// cut, so there are no atomics), then claims chunks of a tail pool as the
// main kernel does.  Every step issues the same vector-memory instructions
// (next packet's descriptors, 4 payload loads, the fold dword, one store --
// to a dummy word when no packet ends) so that the compiler's vmcnt waits are
// exact on every path: a wait merged over paths of different counts would
// stall on loads issued a moment earlier.

constexpr uint32_t UO_PK = 48; // planning charge per record (units = 16-byte pieces)
#ifndef PK_SCHED_BARRIER
#define PK_SCHED_BARRIER 1 // slots folded one after the other (keeps the kernel within 80 VGPRs)
#endif
constexpr uint32_t PK_F = 0;   // dword offsets inside the packed kernel's LDS image
constexpr uint32_t PK_TP = ZDBCRC_OFF_TP - ZDBCRC_OFF_F;
constexpr uint32_t PK_WP = ZDBCRC_OFF_WP - ZDBCRC_OFF_F;
constexpr uint32_t PK_LP = ZDBCRC_OFF_LP - ZDBCRC_OFF_F;
static_assert(ZDBCRC_OFF_F % 4 == 0 && ZDBCRC_PK_LDS_DW % 4 == 0, "packed LDS image must be 16-byte granular");

// Row width RW (lanes per record; 16 unless noted): NR = 64 / RW records per
// packet, a slot is 16 RW bytes of a row's record, a superstep PPS = K RW
// pieces (64 RW bytes).  RW = 8 / 4 read their slot and advance tables from
// TE/WE, TQ/WQ (copied into the TP/WP places of the LDS image) and place lane
// l with LP's column 16 - RW + l.
template <int RW>
struct PkRow {
    static constexpr uint32_t NR = 64 / RW;
    static constexpr uint32_t PPS = K * RW;
    static_assert(RW == 4 || RW == 8 || RW == 16 || RW == 32, "row width");
};

// one row's record in the current packet (uniform within the row)
struct PkGeo {
    uint64_t pb; // Ep - 1024 S + 16 l16: this lane's load address in superstep 0, slot 0
    int32_t kb;  // 64 S - np: positions before it are empty
    uint32_t fl; // lo0 | h << 4 | d << 8 | (Ep & 3) << 16
    uint32_t y;  // the row's fold dword (vector-loaded metadata only; else PkPacket::y)
};
// the packet (wave-uniform)
struct PkPacket {
    uint64_t r0;  // record of row 0 (row g: r0 + g)
    uint32_t nr;  // rows holding a record (1..NR)
    uint32_t S;   // supersteps
    int32_t kmin; // smallest kb of the rows: slots wholly before it are empty
    int32_t kmax; // largest kb: supersteps wholly after it need no edge checks
    bool anyh;    // some row folds bytes
    bool anyd;    // some row loads piece 0 the rare way
    uint32_t y[4]; // each row's fold dword (scalar loads)
};

// per-row scalars -> this lane's row's value
__device__ __forceinline__ uint32_t row_pick(uint32_t lane, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const uint32_t g = lane >> 4;
    return g == 0 ? a : g == 1 ? b : g == 2 ? c : d;
}
__device__ __forceinline__ __attribute__((unused)) uint64_t row_pick64(uint32_t lane, uint64_t a, uint64_t b, uint64_t c,
                                                                       uint64_t d) {
    const uint32_t g = lane >> 4;
    return g == 0 ? a : g == 1 ? b : g == 2 ? c : d;
}

// descriptors of a packet's four rows (records r .. r + 3, clamped to the
// batch).  VM = false: through the scalar cache (no vector registers, no
// vector-memory instructions -- but scalar loads share lgkmcnt with the LDS
// lookups, so the first lookup after them waits out their whole round trip).
// VM = true: one vector load per field, lane l holding row l / 16's
// descriptor (the 16 lanes of a row load one address), completed in order
// with the payload loads they are issued beside.
template <bool VM>
struct PkMeta {
    uint64_t o[4];
    uint32_t l[4];
};
template <>
struct PkMeta<true> {
    uint64_t o;
    uint32_t l;
};
template <bool VM, int RW = 16>
__device__ __forceinline__ void pk_meta(PkMeta<VM> &m, const uint64_t *__restrict__ offsets,
                                        const uint32_t *__restrict__ lengths, uint64_t r, uint64_t n,
                                        uint32_t lane) {
    static_assert(VM || RW == 16, "scalar descriptors: rows of 16 only");
    if constexpr (VM) {
        const uint64_t rg = r + lane / RW;
        const uint64_t i = rg < n ? rg : n - 1;
        m.o = offsets[i];
        m.l = lengths[i];
    } else {
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const uint64_t i = r + g < n ? r + g : n - 1;
            m.o[g] = offsets[i];
            m.l[g] = lengths[i];
        }
    }
}
// this lane's row's descriptor
template <bool VM>
__device__ __forceinline__ uint64_t pk_addr(const PkMeta<VM> &m, uint64_t ab, uint32_t lane) {
    if constexpr (VM)
        return ab + m.o;
    else
        return ab + row_pick64(lane, m.o[0], m.o[1], m.o[2], m.o[3]);
}
template <bool VM>
__device__ __forceinline__ uint32_t pk_len(const PkMeta<VM> &m, uint32_t lane) {
    if constexpr (VM)
        return m.l;
    else
        return row_pick(lane, m.l[0], m.l[1], m.l[2], m.l[3]);
}


__device__ __forceinline__ uint32_t max4rows(uint32_t v) {
    const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    const uint32_t x = a > b ? a : b, y = c > d ? c : d;
    return x > y ? x : y;
}
// the largest of a row-uniform value over the wave's rows of RW lanes: DPP
// row rotations fold the rows of a 16-lane DPP row, then four readlanes
template <int RW>
__device__ __forceinline__ uint32_t max_rows(uint32_t v) {
    if constexpr (RW == 32) {
        const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 32);
        return a > b ? a : b;
    }
    if constexpr (RW <= 4) {
        const uint32_t t = __builtin_amdgcn_update_dpp(0u, v, 0x124, 0xF, 0xF, false); // row_ror:4
        v = t > v ? t : v;
    }
    if constexpr (RW <= 8) {
        const uint32_t t = __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xF, 0xF, false); // row_ror:8
        v = t > v ? t : v;
    }
    return max4rows(v);
}

// geometry of the packet whose row g holds record rg = r0 + g (A, L: its
// descriptor; rows at or past rb are empty), and each row's fold dword
// (scalar loads).  A row without pieces (L - h = 0) gets its grid on the
// table image (`dummy`), so that the loads of its empty positions -- which
// read piece 0's address, F0 = pb + 16 (kb - l16) -- stay inside mapped memory
// even for an empty record at the very end of the arena.
// bit of PkGeo::fl: the row holds no record of this kernel (past the range,
// or a record of the main kernel in a split batch): nothing is stored
constexpr uint32_t PK_NOSTORE = 1u << 24;
template <bool VM, int RW = 16>
__device__ __forceinline__ void pk_geometry(uint64_t A, uint32_t L, uint64_t r0, uint64_t rb, uint32_t lane,
                                            const uint32_t *dummy, uint32_t cls_max, PkGeo &g, PkPacket &p) {
    using R = PkRow<RW>;
    const uint64_t rg = r0 + lane / RW;
    const bool valid = rg < rb && (cls_max == 0 || L <= cls_max);
    if (!valid)
        L = 0;
    const uint64_t E = A + L;
    const uint32_t e3 = (uint32_t)E & 3u;
    const uint32_t h = e3 < L ? e3 : L;
    const uint64_t Ep = E - h;
    const uint32_t Lp = L - h;
    const uint32_t np = (Lp + 15u) >> 4;
    const uint32_t lo0 = 16u * np - Lp;
    uint32_t S = max_rows<RW>((np + R::PPS - 1u) / R::PPS);
    S = S ? S : 1u;
    const int32_t kb = (int32_t)(R::PPS * S) - (int32_t)np;
    const uint32_t kbu = (uint32_t)kb; // kb in [0, 64 S]: compare as unsigned
    p.r0 = r0;
    p.nr = rb - r0 < R::NR ? (uint32_t)(rb - r0) : R::NR;
    p.S = S;
    p.kmax = (int32_t)max_rows<RW>(kbu);
    p.kmin = (int32_t)(~max_rows<RW>(~kbu));
    const uint64_t F0 = Ep - 16ull * np;
    const uint64_t fa = A & ~15ull;
    const uint32_t d = (np && F0 < fa && (fa & 4095ull) == 0) ? (uint32_t)(fa - F0) : 0u;
    p.anyh = __ballot(h != 0) != 0;
    p.anyd = __ballot(d != 0) != 0;
    const uint64_t ya = h ? (Ep & ~3ull) : reinterpret_cast<uint64_t>(dummy);
    if constexpr (VM) {
        g.y = ld_global_u32(ya); // a vector load, in order with the payload's
    } else {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const uint64_t a = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(ya >> 32), 16 * r) << 32) |
                               (uint32_t)__builtin_amdgcn_readlane((uint32_t)ya, 16 * r);
            p.y[r] = ld_global_u32(a);
        }
    }
    const uint64_t Eg = np ? Ep : reinterpret_cast<uint64_t>(dummy); // then F0 = the table image
    g.pb = Eg - 16ull * R::PPS * S + 16ull * (lane % RW);
    g.kb = kb;
    g.fl = lo0 | (h << 4) | (d << 8) | (((uint32_t)Ep & 3u) << 16) | (valid ? 0u : PK_NOSTORE);
}

// piece 0 of a row: the rare shifted load (d: the block holding A, moved up
// by d bytes), then the lo0 bytes before the record cleared
__device__ __forceinline__ uint4 pk_shift_up(uint4 v, uint32_t d) {
    const uint64_t lo = ((uint64_t)v.y << 32) | v.x, hi = ((uint64_t)v.w << 32) | v.z;
    uint64_t nlo, nhi;
    if (d >= 8) {
        nhi = lo << (8u * (d - 8u));
        nlo = 0;
    } else {
        nhi = (hi << (8u * d)) | (lo >> (64u - 8u * d));
        nlo = lo << (8u * d);
    }
    return make_uint4((uint32_t)nlo, (uint32_t)(nlo >> 32), (uint32_t)nhi, (uint32_t)(nhi >> 32));
}

template <bool UNSAFE>
__device__ __forceinline__ uint4 pk_first_piece(uint4 v, uint32_t fl) {
    if (UNSAFE) {
        const uint32_t d = (fl >> 8) & 15u;
        if (d)
            v = pk_shift_up(v, d);
    }
    return mask_piece(v, (int)(fl & 15u), 16);
}

template <bool NTL>
__device__ __forceinline__ uint4 pk_ld(uint64_t a) {
    global_u32x4 *p = reinterpret_cast<global_u32x4 *>(a);
    const u32x4 v = NTL ? __builtin_nontemporal_load(p) : *p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

// the 4 payload loads of superstep s; EDGE: lanes at positions before their
// row's record re-read piece 0 (pk_superstep zeroes them), which comes from
// A's aligned block when it would start in the page below.  No load is
// conditional: a lane that skipped one would keep its register's previous
// value alive.  (CPU model of every address: tests/kernel_model.py
// packed_row_crc, test_packed_loads_stay_in_bounds.)
// TEL (with NTL): the lanes whose 16 bytes reach the 128-byte line holding
// the superstep's last byte load it without the nontemporal hint, so the
// line stays in L2 for the next superstep's first lanes (a record at any byte
// offset shares one line per superstep boundary; TEL 2: also the line of the
// row's first load, which the record before it shares)
template <bool EDGE, bool NTL, int RW = 16, int TEL = 0>
__device__ __forceinline__ void pk_load(uint64_t pb, int32_t kb, uint32_t fl, uint32_t s, uint32_t lane,
                                        uint4 (&buf)[K]) {
    using R = PkRow<RW>;
    const uint64_t base = pb + 16ull * R::PPS * s;
    // piece 0's load address: F0 = Ep - 16 np, moved up to A's aligned block
    // when it would start in the page below (d); the table image for a row
    // without pieces
    const uint64_t F0 = pb + (int64_t)16 * ((int64_t)kb - (int64_t)(lane % RW)) + ((fl >> 8) & 15u);
#pragma unroll
    for (int i = 0; i < K; i++) {
        uint64_t a = base + 16u * RW * i;
        if (EDGE) {
            const int32_t k = (int32_t)(R::PPS * s + RW * i + (lane % RW)) - kb;
            a = k <= 0 ? F0 : a; // k == 0: F0 is piece 0 itself (or its safe block)
        }
        if constexpr (NTL && TEL > 0) {
            bool t = false;
            if (i == K - 1)
                t = ((a + 15) >> 7) == ((base + 16u * R::PPS - 1) >> 7);
            if (TEL > 1 && i == 0)
                t = s == 0 && (a >> 7) == (base >> 7);
            if (t)
                buf[i] = pk_ld<false>(a);
            else
                buf[i] = pk_ld<true>(a);
        } else {
            buf[i] = pk_ld<NTL>(a);
        }
    }
}

// superstep s of the packet folded into the lane register
template <bool EDGE, bool UNSAFE, int RW = 16>
__device__ __forceinline__ uint32_t pk_superstep(const PkGeo &g, const PkPacket &p, uint32_t acc, const uint4 (&cur)[K],
                                                 uint32_t s, uint32_t lane, const uint32_t *lds) {
    if (s)
        acc = advance_superstep_at<PK_WP>(acc, lds);
#define ZDBCRC_PK_SLOT(I)                                                                           \
    if (!EDGE) {                                                                                    \
        acc ^= piece_contrib<I, 0, PK_TP>(cur[I], lds);                                             \
    } else if ((int32_t)(PkRow<RW>::PPS * s + RW * (I) + RW - 1) >= p.kmin) { /* not empty in every row */ \
        const int32_t k = (int32_t)(PkRow<RW>::PPS * s + RW * (I) + (lane % RW)) - g.kb;           \
        uint4 v = cur[I];                                                                           \
        if (k < 0)                                                                                  \
            v = make_uint4(0, 0, 0, 0);                                                             \
        else if (k == 0)                                                                            \
            v = pk_first_piece<UNSAFE>(v, g.fl);                                                    \
        acc ^= piece_contrib<I, 0, PK_TP>(v, lds);                                                  \
    }                                                                                               \
    if (PK_SCHED_BARRIER)                                                                           \
        __builtin_amdgcn_sched_barrier(0);
    ZDBCRC_PK_SLOT(0)
    ZDBCRC_PK_SLOT(1)
    ZDBCRC_PK_SLOT(2)
    ZDBCRC_PK_SLOT(3)
#undef ZDBCRC_PK_SLOT
    return acc;
}

// the packet's crcs: lane placement in the row, DPP reduction over the row,
// fold of the h bytes after the grid (every lane of a row ends with its crc)
template <bool VM, int RW = 16>
__device__ __forceinline__ uint32_t pk_finish(const PkGeo &g, const PkPacket &p, uint32_t acc, uint32_t lane,
                                              const uint32_t *lds) {
    // LP column 16 - RW + (lane mod RW) holds the shift by 16 (RW - 1 - lane mod RW)
    // (rows of 16: column lane & 31, one bank per lane; narrower rows share
    // columns -- a 4-way conflict for rows of 4, once per packet); rows of 32
    // have LT in LP's place, column lane & 31
    const uint32_t col = RW >= 16 ? (lane & 31u) : (16u - RW) + (lane % RW) + (lane & 16u);
    uint32_t x = 0;
#pragma unroll
    for (int c = 0; c < SCH; c++)
        x ^= lds[PK_LP + (c * 32 + ((acc >> (5 * c)) & 31u)) * 32 + col];
    x ^= __builtin_amdgcn_update_dpp(0u, x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    x ^= __builtin_amdgcn_update_dpp(0u, x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    if constexpr (RW == 8)
        x ^= __builtin_amdgcn_update_dpp(0u, x, 0x141, 0xF, 0xF, false); // row_half_mirror
    if constexpr (RW >= 16) {
        x ^= __builtin_amdgcn_update_dpp(0u, x, 0x124, 0xF, 0xF, false); // row_ror:4
        x ^= __builtin_amdgcn_update_dpp(0u, x, 0x128, 0xF, 0xF, false); // row_ror:8
    }
    if constexpr (RW == 32) // the two 16-lane halves of a row
        x ^= __shfl_xor(x, 16, 64);
    if (p.anyh) { // F[0] is the identity: rows without fold bytes pass through
        const uint32_t h = (g.fl >> 4) & 3u;
        const uint32_t y = VM ? g.y : row_pick(lane, p.y[0], p.y[1], p.y[2], p.y[3]);
        x ^= (y >> (8u * ((g.fl >> 16) & 3u))) & ((1u << (8u * h)) - 1u);
        uint32_t r = 0;
#pragma unroll
        for (int c = 0; c < SCH; c++)
            r ^= lds[PK_F + (h * SCH + c) * 32 + ((x >> (5 * c)) & 31u)];
        x = r;
    }
    return x;
}

// first index r in [lo, hi) with f(r) >= key (hi if none); f nondecreasing;
// one vector load per round of the 64-way search
template <class F>
__device__ __forceinline__ uint64_t first_ge(uint64_t lo, uint64_t hi, uint64_t key, uint32_t lane, F f) {
    while (lo < hi) {
        const uint64_t step = (hi - lo + 63) >> 6;
        const uint64_t idx = lo + (uint64_t)lane * step;
        const uint64_t lt = __ballot(idx < hi && f(idx) < key);
        if (!lt)
            return lo;
        const uint32_t L = 63u - (uint32_t)__clzll(lt);
        const uint64_t nhi = lo + (uint64_t)(L + 1) * step;
        lo += (uint64_t)L * step + 1;
        hi = nhi < hi ? nhi : hi;
    }
    return lo;
}

// first record whose first unit is >= key: the block offsets in LDS first
// (boff[b] = unit_start of block b's first record), then the one block
__device__ __forceinline__ uint64_t pk_first_record(const UnitPrefix &us, uint64_t n, uint32_t nb, uint64_t key,
                                                    uint32_t lane) {
    if (!us.boff)
        return first_ge(0, n, key, lane, [&](uint64_t r) { return us.local[r]; });
    const uint64_t b1 = first_ge(0, nb, key, lane, [&](uint64_t b) { return us.boff[b]; });
    if (b1 < nb && us.boff[b1] == key)
        return b1 << us.lg < n ? b1 << us.lg : n;
    const uint64_t b = b1 - 1; // b1 >= 1: boff[0] = 0 <= key
    const uint64_t lo = b << us.lg, hi = ((b + 1) << us.lg) < n ? ((b + 1) << us.lg) : n;
    const uint64_t bo = us.boff[b];
    return first_ge(lo, hi, key, lane, [&](uint64_t r) { return us.local[r] + bo; });
}

// WAITP: 1 = the next superstep's loads are issued once the previous ones
// have landed (one superstep of loads in flight per wave); 0 = two

template <int WGT, int WPE, int DYN = 4, int CPW = 4, uint32_t DYN_POOLS = 32, bool SP = true, int WAITP = 0,
          bool NTL = true, bool VM = false, int RW = 16, bool SB = false, int TEL = 0>
__global__ __launch_bounds__(WGT, WPE) void crc_packed_kernel(
    const uint8_t *__restrict__ arena, const uint64_t *__restrict__ offsets,
    const uint32_t *__restrict__ lengths, const PlanArgs plan, uint64_t n,
    uint32_t *__restrict__ out, const uint32_t *__restrict__ tables, uint32_t max_waves,
    uint32_t *__restrict__ scratch, uint32_t epoch) {
    constexpr uint32_t NW = WGT / 64;
    using R = PkRow<RW>;
    constexpr uint32_t NR = R::NR;
    if (plan.dn) {
        const uint64_t dn = *plan.dn;
        n = dn < n ? dn : n;
    }
    __shared__ __attribute__((aligned(16))) uint32_t lds[ZDBCRC_PK_LDS_DW];
    __shared__ uint64_t boff[PLAN_MAX_BLOCKS + 1];
    __shared__ uint64_t wsum[2 * NW + 1];

    UnitPrefix unit_start{plan.local, nullptr, plan.lg};
    if (plan.bsum) {
        constexpr uint32_t PER = (PLAN_MAX_BLOCKS + WGT - 1) / WGT;
        uint64_t v[PER], t = 0;
#pragma unroll
        for (uint32_t i = 0; i < PER; i++) {
            const uint32_t b = threadIdx.x * PER + i;
            v[i] = b < plan.nb ? plan.bsum[b] : 0;
            t += v[i];
        }
        uint64_t total;
        uint64_t e = block_excl_scan64<WGT>(t, wsum, &total);
#pragma unroll
        for (uint32_t i = 0; i < PER; i++) {
            const uint32_t b = threadIdx.x * PER + i;
            if (b <= plan.nb)
                boff[b] = e;
            e += v[i];
        }
        __syncthreads();
        unit_start.boff = boff;
    }

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gw = __builtin_amdgcn_readfirstlane(blockIdx.x * NW + (threadIdx.x >> 6));
    const uint64_t total = unit_start(n);
    uint64_t nwaves = (total + MIN_UNITS_PER_WAVE - 1) / MIN_UNITS_PER_WAVE;
    if (nwaves > max_waves)
        nwaves = max_waves;
    const bool dyn = DYN > 0 && gridDim.x >= DYN_POOLS && total >= DYN_MIN_UNITS_PER_WAVE * max_waves;
    const uint64_t Ts = dyn ? total - total * DYN / 16 : total;
    const uint32_t *const dummy = tables;
    if (total == 0) { // nothing of this kernel's in the batch (a split batch without small records)
        if (blockIdx.x == 0 && threadIdx.x < DYN_MAX_POOLS)
            scratch[SCRATCH_DYN_CTR + (((epoch + 1u) & 1u) * DYN_MAX_POOLS + threadIdx.x) * 32u] = 0u;
        return;
    }

    // the wave's first range: the records of its static slice (found before
    // the table fill, so that the search's round trips overlap it)
    uint64_t rb = 0, r0 = 0;
    if (gw < nwaves) {
        const uint64_t ub = Ts * gw / nwaves, ue = Ts * (gw + 1) / nwaves;
        if (ub < ue) {
            r0 = pk_first_record(unit_start, n, plan.nb, ub, lane);
            rb = pk_first_record(unit_start, n, plan.nb, ue, lane);
        }
    }
    {
        // the LDS image [F | TP | WP | LP]; narrower rows take their slot and
        // advance tables from TE/WE or TQ/WQ
        constexpr uint32_t TSRC = RW == 32 ? ZDBCRC_OFF_TT : RW == 16 ? ZDBCRC_OFF_TP : RW == 8 ? ZDBCRC_OFF_TE
                                                                                              : ZDBCRC_OFF_TQ;
        constexpr uint32_t WSRC = RW == 32 ? ZDBCRC_OFF_WT : RW == 16 ? ZDBCRC_OFF_WP : RW == 8 ? ZDBCRC_OFF_WE
                                                                                              : ZDBCRC_OFF_WQ;
        constexpr uint32_t LSRC = RW == 32 ? ZDBCRC_OFF_LT : ZDBCRC_OFF_LP;
        static_assert(TSRC % 4 == 0 && WSRC % 4 == 0 && PK_TP % 4 == 0 && PK_WP % 4 == 0 && PK_LP % 4 == 0,
                      "16-byte granular table ranges");
        const uint4 *src = reinterpret_cast<const uint4 *>(tables);
        uint4 *dst = reinterpret_cast<uint4 *>(lds);
        for (uint32_t i = threadIdx.x; i < ZDBCRC_PK_LDS_DW / 4; i += WGT) {
            const uint32_t d = 4 * i;
            const uint32_t sdw = d < PK_TP ? ZDBCRC_OFF_F + d
                                 : d < PK_WP ? TSRC + (d - PK_TP)
                                 : d < PK_LP ? WSRC + (d - PK_WP)
                                             : LSRC + (d - PK_LP);
            dst[i] = src[sdw / 4];
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < DYN_MAX_POOLS) // the next launch's counters (every variant)
        scratch[SCRATCH_DYN_CTR + (((epoch + 1u) & 1u) * DYN_MAX_POOLS + threadIdx.x) * 32u] = 0u;
    __syncthreads();

    // tail pool, as crc_batch_kernel_v3 (pools drawn from every XCD)
    const uint32_t pool = (blockIdx.x + blockIdx.x / DYN_POOLS) % DYN_POOLS;
    const uint64_t Td = total - Ts;
    const uint64_t P0 = Ts + Td * pool / DYN_POOLS;
    const uint64_t PL = Ts + Td * (pool + 1) / DYN_POOLS - P0;
    const uint64_t nch = (uint64_t)CPW * (nwaves / DYN_POOLS);
    uint32_t *const ctr = scratch + SCRATCH_DYN_CTR + ((epoch & 1u) * DYN_MAX_POOLS + pool) * 32u;
    if (SP && dyn)
        __builtin_amdgcn_s_setprio(2);
    uint32_t *const dwave = scratch + gw; // the store of a step without a finished packet

    // Ranges (the static slice, then pool chunks), each walked packet by
    // packet.  Within a range the loads of the next superstep -- this
    // packet's next, or the next packet's first -- are issued before the
    // current one is folded; every step issues the same vector-memory
    // instructions in the same order (fold dword, next descriptors, payload,
    // store), and the next packet's geometry is computed on every step and
    // selected, so the loop carries each value in one place.
    for (;;) {
        if (r0 >= rb) { // next range from the pool
            if (!(DYN && dyn))
                return;
            if (SP)
                __builtin_amdgcn_s_setprio(0);
            for (;;) {
                uint32_t c = 0;
                if (lane == 0)
                    c = atomicAdd(ctr, 1u);
                c = __builtin_amdgcn_readfirstlane(c);
                if (c >= nch)
                    return;
                const uint64_t ub = P0 + PL * c / nch, ue = P0 + PL * (c + 1) / nch;
                if (ue <= ub)
                    continue;
                r0 = pk_first_record(unit_start, n, plan.nb, ub, lane);
                rb = pk_first_record(unit_start, n, plan.nb, ue, lane);
                if (r0 < rb)
                    break;
            }
        }
        // descriptors of the range's first packet, then its geometry
        PkMeta<VM> m;
        pk_meta<VM, RW>(m, offsets, lengths, r0, n, lane);
        const uint64_t ab = reinterpret_cast<uint64_t>(arena);
        PkGeo gc;
        PkPacket pc;
        pk_geometry<VM, RW>(pk_addr<VM>(m, ab, lane), pk_len<VM>(m, lane), r0, rb, lane, dummy, plan.cls_max, gc, pc);
        uint4 cur[K], nxt[K];
        // the loads of superstep s of packet (g, p); with its first superstep,
        // the descriptors of the packet after it (scalar)
        auto issue = [&](const PkGeo &g, PkPacket &p, uint32_t s, uint4(&buf)[K]) {
            if (s == 0)
                pk_meta<VM, RW>(m, offsets, lengths, p.r0 + NR, n, lane);
            if ((int32_t)(R::PPS * s) > p.kmax)
                pk_load<false, NTL, RW, TEL>(g.pb, g.kb, g.fl, s, lane, buf);
            else
                pk_load<true, NTL, RW, TEL>(g.pb, g.kb, g.fl, s, lane, buf);
        };
        issue(gc, pc, 0, cur);
        uint32_t css = 0, acc = 0;
        if constexpr (SB) {
            // one load buffer: a wave folds a superstep, then issues the
            // next one's loads (the other waves of its SIMD cover the wait);
            // 16 + 5 VGPRs fewer than the double-buffered loop below
            for (;;) {
                const bool newp = css + 1 == pc.S;
                const bool last = newp && pc.r0 + NR >= rb;
                if ((int32_t)(R::PPS * css) > pc.kmax)
                    acc = pk_superstep<false, false, RW>(gc, pc, acc, cur, css, lane, lds);
                else if (pc.anyd)
                    acc = pk_superstep<true, true, RW>(gc, pc, acc, cur, css, lane, lds);
                else
                    acc = pk_superstep<true, false, RW>(gc, pc, acc, cur, css, lane, lds);
                uint32_t *dst = dwave;
                uint32_t x = 0;
                if (newp) {
                    x = pk_finish<VM, RW>(gc, pc, acc, lane, lds);
                    acc = 0;
                    if (lane / RW < pc.nr && !(gc.fl & PK_NOSTORE))
                        dst = out + pc.r0 + lane / RW;
                }
                if (lane % RW == 0)
                    *dst = x;
                if (last)
                    break;
                if (newp) {
                    const uint64_t rn = pc.r0 + NR;
                    pk_geometry<VM, RW>(pk_addr<VM>(m, ab, lane), pk_len<VM>(m, lane), rn, rb, lane, dummy,
                                        plan.cls_max, gc, pc);
                    css = 0;
                } else {
                    css++;
                }
                issue(gc, pc, css, cur);
            }
            r0 = rb;
            continue;
        }
        for (;;) {
            const bool newp = css + 1 == pc.S;
            const bool last = newp && pc.r0 + NR >= rb; // the range ends with this packet
            PkGeo gn;
            PkPacket pn;
            const uint32_t nss = newp ? 0u : css + 1;
            if (!last) {
                if (WAITP)
                    __builtin_amdgcn_s_waitcnt(0x0F70);
                if (newp) {
                    pk_geometry<VM, RW>(pk_addr<VM>(m, ab, lane), pk_len<VM>(m, lane), pc.r0 + NR, rb, lane, dummy,
                                        plan.cls_max, gn, pn);
                    issue(gn, pn, 0, nxt);
                } else {
                    issue(gc, pc, nss, nxt);
                }
            }
            if ((int32_t)(R::PPS * css) > pc.kmax)
                acc = pk_superstep<false, false, RW>(gc, pc, acc, cur, css, lane, lds);
            else if (pc.anyd)
                acc = pk_superstep<true, true, RW>(gc, pc, acc, cur, css, lane, lds);
            else
                acc = pk_superstep<true, false, RW>(gc, pc, acc, cur, css, lane, lds);
            uint32_t *dst = dwave;
            uint32_t x = 0;
            if (newp) {
                x = pk_finish<VM, RW>(gc, pc, acc, lane, lds);
                acc = 0;
                if (lane / RW < pc.nr && !(gc.fl & PK_NOSTORE))
                    dst = out + pc.r0 + lane / RW;
            }
            if (lane % RW == 0)
                *dst = x;
            if (last)
                break;
            if (newp) {
                gc = gn;
                pc = pn;
            }
            css = nss;
#pragma unroll
            for (int i = 0; i < K; i++)
                cur[i] = nxt[i];
        }
        r0 = rb; // range done
    }
}

typedef void (*crc_kernel_fn)(const uint8_t *, const uint64_t *, const uint32_t *, PlanArgs, uint64_t,
                              uint32_t *, const uint32_t *, uint32_t, uint32_t *, uint32_t);

struct KernelVariant {
    const char *name;
    crc_kernel_fn fn;
    int threads;
    int wgs_per_cu = WG_PER_CU;
    uint32_t unit_ovh = UNIT_OVH; // must match the kernel's UO
};

// batches of records <= 4 KiB: the packed kernel with vector-loaded
// descriptors and fold dwords and ONE load buffer -- a wave
// folds a superstep, then issues the next one's loads; the other waves of its
// SIMD cover the wait.  That brought it to 74 VGPRs and 768 threads (6 waves
// per SIMD; the double-buffered 512-thread form ran 4): fixed 4 KiB 0.798 ->
// 0.709 ms, Zipf <= 2 KiB 2.70 -> 2.31 (profiles/r3/ab_packed_single_buffer.jsonl).
// Squeezed to 64 VGPRs for 1024 threads (8 waves per SIMD) it gains another
// 1-8 % on every shape and bound measured (profiles/r3/ab_packed_8waves*.jsonl).
const KernelVariant kTiny = {"pk_wg1024_dyn4c4p32_sp_vm_sb",
                             crc_packed_kernel<1024, 8, 4, 4, 32, true, 0, true, true, 16, true>, 1024, WG_PER_CU,
                             UO_PK};
const KernelVariant kTiny8 = {"pk8_wg1024_dyn4c4p32_sp_vm_sb",
                              crc_packed_kernel<1024, 8, 4, 4, 32, true, 0, true, true, 8, true>, 1024, WG_PER_CU,
                              UO_PK};
const KernelVariant kTiny4 = {"pk4_wg1024_dyn4c4p32_sp_vm_sb",
                              crc_packed_kernel<1024, 8, 4, 4, 32, true, 0, true, true, 4, true>, 1024, WG_PER_CU,
                              UO_PK};

// Diagnostic library only (A/B): a batch without a known bound split by
// record size -- records of at most `split` bytes to the packed kernel, the
// rest to the main kernel, planned in one planner launch (two unit prefixes,
// a record has units in one of them) and run back to back on the stream.
// Measured and not shipped: C3's main kernel gets 1.8 %
// faster without its 57,822 records of <= 1 KiB, but their packed launch
// takes 39 us and the step goes 0.727 -> 0.749 ms
// (profiles/r3/ab_split_small_records.jsonl).
const KernelVariant &split_variant(uint32_t split) {
    return split <= TINY4_RECORD_MAX ? kTiny4 : split <= TINY8_RECORD_MAX ? kTiny8 : kTiny;
}

#ifdef ZDBCRC_DIAG
// diagnostic library only (libzdbcrc_diag.so, scripts/ab.py): A/B variants,
// several of which compute wrong checksums by design (NOZ, NOLOAD, XM);
// selectable with ZDBCRC_VARIANT=<index> or zdbcrc_debug_set_variant
const KernelVariant kVariants[] = {
    {"v3_wg768_nt_dyn4c4p32_sp_xp", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true, 0, false, false, true>, 768},
    {"v3_wg768_nt_dyn6c4p32", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 6, 4, 32>, 768},
    {"v3_wg768_prio_nt", crc_batch_kernel_v3<768, 6, false, 1, UNIT_OVH, false, true>, 768},
    {"v3_wg768_prio", crc_batch_kernel_v3<768, 6, false, 1>, 768},
    {"v3_wg768_nt", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true>, 768},
    {"v3_wg768_prio_nt_stamp", crc_batch_kernel_v3<768, 6, true, 1, UNIT_OVH, false, true>, 768},
    {"v3_wg768_prio_nt_noz", crc_batch_kernel_v3<768, 6, false, 1, UNIT_OVH, true, true>, 768},
    {"v3_wg768_prio_noload", crc_batch_kernel_v3<768, 6, false, 1, UNIT_OVH, false, true, true>, 768},
    {"v3_wg768_prio_nt_cheapx", crc_batch_kernel_v3<768, 6, false, 1, UNIT_OVH, false, true, false, 1>, 768},
    {"v3_wg1024_prio_nt", crc_batch_kernel_v3<1024, 8, false, 1, UNIT_OVH, false, true>, 1024},
    {"v3_wg768_prio_nt_a16", crc_batch_kernel_v3<768, 6, false, 1, UNIT_OVH, false, true, false, 3>, 768},
    {"v3_wg768_prio_noload_a16", crc_batch_kernel_v3<768, 6, false, 1, UNIT_OVH, false, true, true, 3>, 768},
    {"v3_wg768_prio_noload_cheapx", crc_batch_kernel_v3<768, 6, false, 1, UNIT_OVH, false, true, true, 1>, 768},
    {"v3_wg1024_prio_noload", crc_batch_kernel_v3<1024, 8, false, 1, UNIT_OVH, false, true, true>, 1024},
    {"v3_wg512_prio_noload", crc_batch_kernel_v3<512, 4, false, 1, UNIT_OVH, false, true, true>, 512},
    {"v3_wg512_prio_nt", crc_batch_kernel_v3<512, 4, false, 1, UNIT_OVH, false, true>, 512},
    {"v3_wg768_prio2_nt", crc_batch_kernel_v3<768, 6, false, 2, UNIT_OVH, false, true>, 768},
    {"v3_wg768_prio3_nt", crc_batch_kernel_v3<768, 6, false, 3, UNIT_OVH, false, true>, 768},
    {"v3_wg768_prio2_nt_stamp", crc_batch_kernel_v3<768, 6, true, 2, UNIT_OVH, false, true>, 768},
    {"v3_wg768_prio3_nt_stamp", crc_batch_kernel_v3<768, 6, true, 3, UNIT_OVH, false, true>, 768},
    {"v3_wg768_nt_dyn8c3p32", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 8, 3, 32>, 768},
    {"v3_wg768_nt_dyn6c4p32_uo768", crc_batch_kernel_v3<768, 6, false, 0, 768, false, true, false, 0, 6, 4, 32>, 768, WG_PER_CU, 768},
    {"v3_wg768_nt_dyn4c4p32", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32>, 768},
    {"v3_wg768_nt_dyn4c4p32_sp_stamp", crc_batch_kernel_v3<768, 6, true, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true>, 768},
    {"v3_wg768_nt_dyn4c4p32_sp_noload", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, true, 0, 4, 4, 32, true>, 768},
    {"v3_wg768_nt_dyn4c4p32_sp_pp", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true, 1>, 768},
    {"v3_wg768_nt_dyn4c4p32_sp_pp_wait", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true, 3>, 768},
    {"v3_wg768_nt_dyn4c4p32_sp_noz", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, 1, true, false, 0, 4, 4, 32, true>, 768},
    {"v3_wg768_nt_dyn4c4p32_sp_noz_noplace", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, 2, true, false, 0, 4, 4, 32, true>, 768},
    // debugging: the default kernel writing each wave's last segment (pa, pb, value, r | np << 32)
    {"v3_wg768_nt_dyn4c4p32_sp_segdump", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true, 0, true>, 768},
    // round 2: the record-relative grid on byte-misaligned loads (BMG, the previous default) against the
    // default's loads from the dword below the record
    {"v3_wg768_nt_dyn4c4p32_sp_bmg", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true, 0, false, true>, 768},
    {"v3_wg768_nt_dyn4c4p32_sp_pp_wait_bmg", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true, 3, false, true>, 768},
    // round 2: tail pools drawn from every XCD (XP; index 0 is the product default with XP, this
    // the default before it)
    {"v3_wg768_nt_dyn4c4p32_sp", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true>, 768},
    {"v3_wg768_nt_dyn4c4p32_sp_pp_wait_bmg_xp", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true, 3, false, true, true>, 768},
    {"v3_wg768_nt_dyn4c4p32_sp_stamp_xp", crc_batch_kernel_v3<768, 6, true, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true, 0, false, false, true>, 768},
    // round 2: pool share and chunks per wave re-checked with the XCD pools
    {"v3_wg768_nt_dyn3c4p32_sp_xp", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 3, 4, 32, true, 0, false, false, true>, 768},
    {"v3_wg768_nt_dyn5c4p32_sp_xp", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 5, 4, 32, true, 0, false, false, true>, 768},
    {"v3_wg768_nt_dyn4c3p32_sp_xp", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 3, 32, true, 0, false, false, true>, 768},
    // round 2, after the dword grid: planning charge and pool share re-checked
    {"v3_wg768_nt_dyn4c4p32_sp_uo256", crc_batch_kernel_v3<768, 6, false, 0, 256, false, true, false, 0, 4, 4, 32, true>, 768, WG_PER_CU, 256},
    {"v3_wg768_nt_dyn4c4p32_sp_uo512", crc_batch_kernel_v3<768, 6, false, 0, 512, false, true, false, 0, 4, 4, 32, true>, 768, WG_PER_CU, 512},
    {"v3_wg768_nt_dyn3c4p32_sp", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 3, 4, 32, true>, 768},
    {"v3_wg768_nt_dyn5c4p32_sp", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 5, 4, 32, true>, 768},
    // round 3: the packed small-record kernel (four records per wave, one per row of 16 lanes)
    {"pk_wg768_dyn4c4p32_sp", crc_packed_kernel<768, 6, 4, 4, 32, true, 0>, 768, WG_PER_CU, UO_PK},
    {"pk_wg768_dyn4c4p32_sp_wait", crc_packed_kernel<768, 6, 4, 4, 32, true, 1>, 768, WG_PER_CU, UO_PK},
    {"pk_wg640_dyn4c4p32_sp", crc_packed_kernel<640, 5, 4, 4, 32, true, 0>, 640, WG_PER_CU, UO_PK},
    {"pk_wg640_dyn4c4p32_sp_wait", crc_packed_kernel<640, 5, 4, 4, 32, true, 1>, 640, WG_PER_CU, UO_PK},
    {"pk_wg512_dyn4c4p32_sp", crc_packed_kernel<512, 4, 4, 4, 32, true, 0>, 512, WG_PER_CU, UO_PK},
    // round 3 (resumed): descriptors and fold dwords as vector loads (no scalar-load waits per packet)
    {"pk_wg512_dyn4c4p32_sp_vm", crc_packed_kernel<512, 4, 4, 4, 32, true, 0, true, true>, 512, WG_PER_CU, UO_PK},
    {"pk_wg768_dyn4c4p32_sp_vm", crc_packed_kernel<768, 6, 4, 4, 32, true, 0, true, true>, 768, WG_PER_CU, UO_PK},
    {"pk_wg512_dyn4c4p32_sp_wait_vm", crc_packed_kernel<512, 4, 4, 4, 32, true, 1, true, true>, 512, WG_PER_CU, UO_PK},
    {"pk_wg640_dyn4c4p32_sp_wait_vm", crc_packed_kernel<640, 5, 4, 4, 32, true, 1, true, true>, 640, WG_PER_CU, UO_PK},
    {"pk_wg768_dyn4c4p32_sp_wait_vm", crc_packed_kernel<768, 6, 4, 4, 32, true, 1, true, true>, 768, WG_PER_CU, UO_PK},
    // round 3 (resumed): the dword grid for record-relative records of every size, now that its fold dword
    // is a global (not flat) load -- small shape and default
    {"v3_wg768_nt_dyn4c4p32_sp_pp_wait_dwg0_xp", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true, 3, false, false, true, 0>, 768},
    {"v3_wg768_nt_dyn4c4p32_sp_dwg0_xp", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true, 0, false, false, true, 0>, 768},
    // round 3 (resumed): record search through the planner's blocks (one HBM round trip per search)
    {"v3_wg768_nt_dyn4c4p32_sp_xp_frb", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true, 0, false, false, true, DWG_MIN_BYTES, true>, 768},
    {"v3_wg768_nt_dyn4c4p32_sp_pp_wait_bmg_xp_frb", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true, 3, false, true, true, DWG_MIN_BYTES, true>, 768},
    // rows of 8 and 4 lanes (8 / 16 records per wave)
    {"pk8_wg512_dyn4c4p32_sp_wait_vm", crc_packed_kernel<512, 4, 4, 4, 32, true, 1, true, true, 8>, 512, WG_PER_CU, UO_PK},
    {"pk4_wg512_dyn4c4p32_sp_wait_vm", crc_packed_kernel<512, 4, 4, 4, 32, true, 1, true, true, 4>, 512, WG_PER_CU, UO_PK},
    {"pk8_wg512_dyn4c4p32_sp_vm", crc_packed_kernel<512, 4, 4, 4, 32, true, 0, true, true, 8>, 512, WG_PER_CU, UO_PK},
    {"pk4_wg512_dyn4c4p32_sp_vm", crc_packed_kernel<512, 4, 4, 4, 32, true, 0, true, true, 4>, 512, WG_PER_CU, UO_PK},
    // single load buffer (fold, then issue the next loads): fits 6 waves per SIMD
    {"pk_wg768_dyn4c4p32_sp_vm_sb", crc_packed_kernel<768, 6, 4, 4, 32, true, 0, true, true, 16, true>, 768, WG_PER_CU, UO_PK},
    {"pk8_wg768_dyn4c4p32_sp_vm_sb", crc_packed_kernel<768, 6, 4, 4, 32, true, 0, true, true, 8, true>, 768, WG_PER_CU, UO_PK},
    {"pk_wg512_dyn4c4p32_sp_vm_sb", crc_packed_kernel<512, 4, 4, 4, 32, true, 0, true, true, 16, true>, 512, WG_PER_CU, UO_PK},
    {"pk4_wg768_dyn4c4p32_sp_vm_sb", crc_packed_kernel<768, 6, 4, 4, 32, true, 0, true, true, 4, true>, 768, WG_PER_CU, UO_PK},
    // round 3 (resumed): one load buffer (the next superstep's loads after the fold), more waves per SIMD
    {"v3_wg1024_nt_dyn4c4p32_sp_xp_sb", crc_batch_kernel_v3<1024, 8, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true, 0, false, false, true, DWG_MIN_BYTES, false, true>, 1024},
    {"v3_wg768_nt_dyn4c4p32_sp_xp_sb", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true, 0, false, false, true, DWG_MIN_BYTES, false, true>, 768},
    // one-buffer packed kernel with plain (temporal) payload loads: a row's segments share lines at their edges
    {"pk_wg768_dyn4c4p32_sp_vm_sb_tl", crc_packed_kernel<768, 6, 4, 4, 32, true, 0, false, true, 16, true>, 768, WG_PER_CU, UO_PK},
    {"pk8_wg768_dyn4c4p32_sp_vm_sb_tl", crc_packed_kernel<768, 6, 4, 4, 32, true, 0, false, true, 8, true>, 768, WG_PER_CU, UO_PK},
    // one-buffer packed kernel at 8 waves per SIMD (1024-thread workgroups, <= 64 VGPRs)
    {"pk_wg1024_dyn4c4p32_sp_vm_sb", crc_packed_kernel<1024, 8, 4, 4, 32, true, 0, true, true, 16, true>, 1024, WG_PER_CU, UO_PK},
    {"pk8_wg1024_dyn4c4p32_sp_vm_sb", crc_packed_kernel<1024, 8, 4, 4, 32, true, 0, true, true, 8, true>, 1024, WG_PER_CU, UO_PK},
    {"pk4_wg1024_dyn4c4p32_sp_vm_sb", crc_packed_kernel<1024, 8, 4, 4, 32, true, 0, true, true, 4, true>, 1024, WG_PER_CU, UO_PK},
    {"pk_wg1024_dyn4c4p32_sp_vm_sb_tel1", crc_packed_kernel<1024, 8, 4, 4, 32, true, 0, true, true, 16, true, 1>, 1024, WG_PER_CU, UO_PK},
    {"pk_wg1024_dyn4c4p32_sp_vm_sb_tel2", crc_packed_kernel<1024, 8, 4, 4, 32, true, 0, true, true, 16, true, 2>, 1024, WG_PER_CU, UO_PK},
    {"pk8_wg1024_dyn4c4p32_sp_vm_sb_tel1", crc_packed_kernel<1024, 8, 4, 4, 32, true, 0, true, true, 8, true, 1>, 1024, WG_PER_CU, UO_PK},
    // rows of 32 lanes (two records per wave)
    {"pk32_wg768_dyn4c4p32_sp_vm_sb", crc_packed_kernel<768, 6, 4, 4, 32, true, 0, true, true, 32, true>, 768, WG_PER_CU, UO_PK},

    {"v3_wg768_nt_dyn4c4p32_sp_xp_tel1", crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true, 0, false, false, true, DWG_MIN_BYTES, false, false, 1>, 768},
    {"pk_wg1024_dyn6c4p32_sp_vm_sb", crc_packed_kernel<1024, 8, 6, 4, 32, true, 0, true, true, 16, true>, 1024, WG_PER_CU, UO_PK},
    {"pk_wg1024_dyn4c2p32_sp_vm_sb", crc_packed_kernel<1024, 8, 4, 2, 32, true, 0, true, true, 16, true>, 1024, WG_PER_CU, UO_PK},
    {"pk_wg1024_dyn2c4p32_sp_vm_sb", crc_packed_kernel<1024, 8, 2, 4, 32, true, 0, true, true, 16, true>, 1024, WG_PER_CU, UO_PK},
    {"pk_wg1024_dyn4c4p8_sp_vm_sb", crc_packed_kernel<1024, 8, 4, 4, 8, true, 0, true, true, 16, true>, 1024, WG_PER_CU, UO_PK},
    {"v3_wg1024_nt_dyn4c4p32_sp_xp", crc_batch_kernel_v3<1024, 8, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true, 0, false, false, true>, 1024},
};
constexpr int kNumVariants = (int)(sizeof(kVariants) / sizeof(kVariants[0]));
std::atomic<int> g_variant{-1};
// A/B: split unbounded batches at this many bytes (0: never; zdbcrc_debug_set_split)
std::atomic<uint32_t> g_debug_split{0};
uint32_t split_bytes(const KernelVariant &) { return g_debug_split.load(); }
std::atomic<int> g_host_mode{0};

const KernelVariant &variant(uint64_t /*max_len: the A/B harness picks by index*/ = 0) {
    int v = g_variant.load();
    if (v < 0) {
        const char *e = std::getenv("ZDBCRC_VARIANT");
        const int i = e ? std::atoi(e) : 0;
        int expect = -1;
        g_variant.compare_exchange_strong(expect, (i >= 0 && i < kNumVariants) ? i : 0);
        v = g_variant.load();
    }
    return kVariants[v];
}
#else
// the product library ships the main checksum kernel (any records; tail
// pool: 4/16 of the units, 32 pools drawn from every XCD, 4 chunks per wave,
// static-phase priority, 768 threads, nontemporal payload loads; DESIGN.md
// §4.1) and the packed kernel for batches known to hold records of at most
// 4 KiB (above), no environment knob.  Every shape is exact for any input;
// the choice only changes speed.
const KernelVariant kDefault = {"v3_wg768_nt_dyn4c4p32_sp_xp",
                                crc_batch_kernel_v3<768, 6, false, 0, UNIT_OVH, false, true, false, 0, 4, 4, 32, true,
                                                    0, false, false, true>,
                                768};
// the product never splits a batch (diagnostic A/B only)
constexpr uint32_t split_bytes(const KernelVariant &) { return 0u; }
// the kernel for a batch whose records are at most max_len bytes (0: unknown)
const KernelVariant &variant(uint64_t max_len = 0) {
    if (max_len == 0 || max_len > TINY_RECORD_MAX)
        return kDefault;
    if (max_len <= TINY4_RECORD_MAX)
        return kTiny4;
    return max_len <= TINY8_RECORD_MAX ? kTiny8 : kTiny;
}
#endif

// unit count per record: ovh (the variant's per-record charge) + number of
// 16-byte pieces it touches
struct UnitCount {
    const uint8_t *arena;
    const uint64_t *offsets;
    const uint32_t *lengths;
    uint64_t n;
    uint64_t ovh;
    __host__ __device__ uint64_t operator()(uint64_t r) const {
        if (r >= n)
            return 0;
        const uint32_t L = lengths[r];
        if (!L)
            return ovh;
        const uint64_t a = reinterpret_cast<uint64_t>(arena) + offsets[r];
        return ovh + record_pieces(a, L);
    }
};

// planner (one launch): every record's unit count, the exclusive prefix
// inside blocks of 2^lg records (local: n + 1 entries, entry n closes the
// last block) and each block's total (bsum); zeroes out[] on the way (cut
// records are finished by atomic XOR).  The checksum kernel scans the <= 1024
// block totals itself, so there is no grid-wide dependency here.
// SPLIT: two plans at once -- records of more than `split` bytes for the main
// kernel (ovh per record), the others for the packed kernel (ovh_s); a
// record has units in one plan only.
constexpr uint32_t PLAN_T = 256;
struct PlanOut {
    uint64_t *local;
    uint64_t *bsum;
    uint32_t *bmax;
};

template <bool SPLIT>
__device__ __forceinline__ uint64_t plan_units(const uint8_t *arena, const uint64_t *offsets, uint32_t L, uint64_t r,
                                               uint64_t ovh, bool mine) {
    if (!mine)
        return 0;
    uint64_t v = ovh;
    if (L) {
        const uint64_t a = reinterpret_cast<uint64_t>(arena) + offsets[r];
        v += record_pieces(a, L);
    }
    return v;
}

template <bool SPLIT>
__global__ __launch_bounds__(PLAN_T) void plan_kernel(const uint8_t *__restrict__ arena,
                                                      const uint64_t *__restrict__ offsets,
                                                      const uint32_t *__restrict__ lengths, uint64_t n, uint64_t ovh,
                                                      uint32_t lg, PlanOut pb, uint32_t *__restrict__ out,
                                                      const uint64_t *__restrict__ dn, uint32_t split, uint64_t ovh_s,
                                                      PlanOut ps) {
    if (dn) { // device-side record count, n its bound (records past it: no units)
        const uint64_t m = *dn;
        n = m < n ? m : n;
    }
    __shared__ uint64_t wsum[2 * (PLAN_T / 64) + 1];
    __shared__ uint32_t wmx[2][PLAN_T / 64];
    uint32_t mx = 0, mxs = 0;
    const uint32_t per = (1u << lg) / PLAN_T;
    const uint64_t r0 = ((uint64_t)blockIdx.x << lg) + (uint64_t)threadIdx.x * per;
    uint64_t s = 0, ss = 0;
    for (uint32_t i = 0; i < per; i++) {
        const uint64_t r = r0 + i;
        if (r < n) {
            const uint32_t L = lengths[r];
            const bool small = SPLIT && L <= split;
            const uint64_t v = plan_units<SPLIT>(arena, offsets, L, r, ovh, !small);
            s += v;
            mx = v > mx ? (uint32_t)v : mx;
            if (SPLIT) {
                const uint64_t vs = plan_units<SPLIT>(arena, offsets, L, r, ovh_s, small);
                ss += vs;
                mxs = vs > mxs ? (uint32_t)vs : mxs;
            }
            out[r] = 0;
        }
    }
    mx = wave_max(mx);
    if (SPLIT)
        mxs = wave_max(mxs);
    if ((threadIdx.x & 63u) == 0) {
        wmx[0][threadIdx.x >> 6] = mx;
        wmx[1][threadIdx.x >> 6] = mxs;
    }
    uint64_t total, total_s = 0;
    uint64_t e = block_excl_scan64<PLAN_T>(s, wsum, &total); // its barriers publish wmx
    uint64_t es = SPLIT ? block_excl_scan64<PLAN_T>(ss, wsum, &total_s) : 0;
    for (uint32_t i = 0; i < per; i++) {
        const uint64_t r = r0 + i;
        if (r > n)
            break;
        pb.local[r] = e;
        if (SPLIT)
            ps.local[r] = es;
        if (r < n) {
            const uint32_t L = lengths[r];
            const bool small = SPLIT && L <= split;
            e += plan_units<SPLIT>(arena, offsets, L, r, ovh, !small);
            if (SPLIT)
                es += plan_units<SPLIT>(arena, offsets, L, r, ovh_s, small);
        }
    }
    if (threadIdx.x == 0) {
        uint32_t m = 0, ms = 0;
        for (uint32_t i = 0; i < PLAN_T / 64; i++) {
            m = wmx[0][i] > m ? wmx[0][i] : m;
            ms = wmx[1][i] > ms ? wmx[1][i] : ms;
        }
        pb.bsum[blockIdx.x] = total;
        pb.bmax[blockIdx.x] = m;
        if (SPLIT) {
            ps.bsum[blockIdx.x] = total_s;
            ps.bmax[blockIdx.x] = ms;
        }
    }
}

__global__ void verify_kernel(const uint32_t *__restrict__ out, const uint32_t *__restrict__ expected,
                              uint64_t n, uint32_t *__restrict__ mismatch, uint32_t *__restrict__ count,
                              uint32_t max_mismatch, const uint64_t *__restrict__ dn) {
    if (dn) {
        const uint64_t m = *dn;
        n = m < n ? m : n;
    }
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n && out[r] != expected[r]) {
        const uint32_t idx = atomicAdd(count, 1u);
        if (idx < max_mismatch)
            mismatch[idx] = (uint32_t)r;
    }
}

// batched CHECK, phase 1: decode the entry header at each index-given offset
// (data_entry_header_t, data.h:56-65: u8 idlength, u32 datalength, u32
// previous, u32 integrity, ...; 18 bytes, packed LE) into checksum
// descriptors.  Records whose header or payload leaves the image get length 0
// and status -1 (data_check_real's short reads, data.c:540-555).
__device__ __forceinline__ uint32_t le32_at(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__global__ void check_decode_kernel(const uint8_t *__restrict__ image, uint64_t image_len,
                                    const uint64_t *__restrict__ rec_off, uint64_t n,
                                    uint64_t *__restrict__ offs, uint32_t *__restrict__ lens,
                                    uint32_t *__restrict__ expect, int32_t *__restrict__ result) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint64_t o = rec_off[i];
    uint64_t po = 0;
    uint32_t len = 0, crc = 0;
    int32_t st = -1;
    if (o <= image_len && image_len - o >= ZDB_ENTRY_HEADER_SIZE) {
        const uint8_t *h = image + o;
        const uint64_t p = o + ZDB_ENTRY_HEADER_SIZE + h[0];
        const uint32_t L = le32_at(h + 1);
        // read(fd, buf, 0) succeeds wherever the file position is, so an
        // empty payload is checked (crc 0 vs integrity) even when the key
        // runs past the end of the image (data.c:546-551)
        if (L == 0 || (p <= image_len && image_len - p >= L)) {
            po = L ? p : 0;
            len = L;
            crc = le32_at(h + 9);
            st = 0;
        }
    }
    offs[i] = po;
    lens[i] = len;
    expect[i] = crc;
    result[i] = st;
}

// phase 2: 1 / 0 from the computed checksums, -1 kept
__global__ void check_finish_kernel(const uint32_t *__restrict__ out, const uint32_t *__restrict__ expect,
                                    uint64_t n, int32_t *__restrict__ result) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && result[i] == 0)
        result[i] = out[i] == expect[i] ? 1 : 0;
}

// end of a small host batch (C5 latency path): one wave moves the results
// into the mailbox (mapped, host-coherent memory), re-zeroes the device
// result buffer for the next batch (so no memset precedes it), and then
// publishes the batch's sequence number with a system-scope release store.
// The host spins on that word: no copy engine, no stream synchronize.  (The
// same work as an epilogue of the checksum kernel -- the last wave to arrive
// on a counter publishes -- measured slower: 17.2 vs 16.0 us for one 64 B
// value, 308 vs 196 us for 8 x 1 MiB, the arrivals being same-address
// atomics; profiles/r2/c5_host_modes.jsonl.)
__global__ __launch_bounds__(64) void publish_kernel(uint32_t *__restrict__ d_out, uint32_t *__restrict__ mbox_out,
                                                      uint32_t n, uint32_t *mbox_seq, uint32_t seq) {
    for (uint32_t i = threadIdx.x; i < n; i += 64) {
        mbox_out[i] = d_out[i];
        d_out[i] = 0;
    }
    __threadfence_system();
    if (threadIdx.x == 0)
        __hip_atomic_store(mbox_seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

#ifdef ZDBCRC_DIAG
// read-only streaming probe (measurement aid): XOR of every 16-byte word,
// one dword written per workgroup -- the achievable HBM read ceiling the
// checksum kernel is compared with
__global__ __launch_bounds__(256) void stream_read_kernel(const uint4 *__restrict__ src, uint64_t words,
                                                          uint32_t *__restrict__ sink) {
    uint4 a = make_uint4(0, 0, 0, 0), b = a, c = a, d = a;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < words; i += 4 * stride) {
        const uint4 x0 = src[i], x1 = src[i + stride], x2 = src[i + 2 * stride], x3 = src[i + 3 * stride];
        a.x ^= x0.x; a.y ^= x0.y; a.z ^= x0.z; a.w ^= x0.w;
        b.x ^= x1.x; b.y ^= x1.y; b.z ^= x1.z; b.w ^= x1.w;
        c.x ^= x2.x; c.y ^= x2.y; c.z ^= x2.z; c.w ^= x2.w;
        d.x ^= x3.x; d.y ^= x3.y; d.z ^= x3.z; d.w ^= x3.w;
    }
    for (; i < words; i += stride) {
        const uint4 x0 = src[i];
        a.x ^= x0.x; a.y ^= x0.y; a.z ^= x0.z; a.w ^= x0.w;
    }
    uint32_t v = a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
    v = wave_xor(v);
    if ((threadIdx.x & 63) == 0)
        atomicXor(sink + blockIdx.x, v);
}

// contiguous-slice variant of the probe: wave w reads its own slice, 1 KiB
// per load instruction, U loads per lane per iteration -- the access shape of
// crc_batch_kernel without any checksum work
// read probe of the packed kernels' access shape: the arena as 4 KiB
// records, a wave walking packets of 64 / RW records, row g (RW lanes) on
// record g of the packet, U loads of RW x 16 B per row in flight (each load
// instruction touches 64 / RW separate RW x 16-byte segments), nontemporal
template <int RW, int U>
__global__ __launch_bounds__(1024) void stream_rows_kernel(const uint4 *__restrict__ src, uint64_t words,
                                                           uint32_t *__restrict__ sink) {
    constexpr uint64_t REC_W = 256, NR = 64 / RW;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const uint64_t npk = words / REC_W / NR;
    const uint64_t lo = npk * w / nw, hi = npk * (w + 1) / nw;
    uint4 a = make_uint4(0, 0, 0, 0);
    for (uint64_t pk = lo; pk < hi; pk++) {
        const uint64_t base = pk * NR * REC_W + (lane / RW) * REC_W + (lane % RW);
        for (uint32_t j = 0; j < REC_W / RW; j += U) {
            uint4 x[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src + base + RW * (j + u)));
                x[u] = make_uint4(t.x, t.y, t.z, t.w);
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                a.x ^= x[u].x; a.y ^= x[u].y; a.z ^= x[u].z; a.w ^= x[u].w;
            }
        }
    }
    uint32_t v = wave_xor(a.x ^ a.y ^ a.z ^ a.w);
    if (lane == 0)
        atomicXor(sink + (w & 0xFFFF), v);
}

template <int U, bool NTL = false>
__global__ __launch_bounds__(1024) void stream_slice_kernel(const uint4 *__restrict__ src, uint64_t words,
                                                            uint32_t *__restrict__ sink) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const uint64_t lo = words * w / nw, hi = words * (w + 1) / nw;
    uint4 a = make_uint4(0, 0, 0, 0);
    uint64_t i = lo + lane;
    for (; i + 64 * (U - 1) < hi; i += 64 * U) {
        uint4 x[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            if (NTL) {
                const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src + i + 64 * u));
                x[u] = make_uint4(t.x, t.y, t.z, t.w);
            } else {
                x[u] = src[i + 64 * u];
            }
#pragma unroll
        for (int u = 0; u < U; u++) {
            a.x ^= x[u].x; a.y ^= x[u].y; a.z ^= x[u].z; a.w ^= x[u].w;
        }
    }
    for (; i < hi; i += 64) {
        const uint4 x0 = src[i];
        a.x ^= x0.x; a.y ^= x0.y; a.z ^= x0.z; a.w ^= x0.w;
    }
    uint32_t v = wave_xor(a.x ^ a.y ^ a.z ^ a.w);
    if (lane == 0)
        atomicXor(sink + (w & 0xFFFF), v);
}

// LDS lookup microbenchmark (measurement aid): every lane does ITERS rounds
// of 16 independent table lookups (5-bit indices from a per-lane xorshift
// state, V VALU ops of index extraction per lookup) into 32-entry tables,
// XOR-folded; B64: ds_read_b64 of 8-byte entries instead of ds_read_b32
template <int V, bool B64>
__global__ __launch_bounds__(768, 6) void lds_bench_kernel(uint32_t iters, uint32_t *__restrict__ sink) {
    __shared__ __attribute__((aligned(16))) uint32_t tab[16 * 64];
    for (int i = threadIdx.x; i < 16 * 64; i += blockDim.x)
        tab[i] = i * 0x9E3779B9u;
    __syncthreads();
    uint32_t x = (blockIdx.x * blockDim.x + threadIdx.x) * 0x85EBCA6Bu + 1u, acc = 0;
    for (uint32_t it = 0; it < iters; it++) {
        uint32_t r = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t w = k < 8 ? x : acc ^ x;
            uint32_t a;
            if (V == 1)
                a = (w >> (4 * (k & 7))) & (B64 ? 0xF8u : 0x7Cu);
            else
                a = ((w >> (3 * (k & 7) + 1)) & 31u) << (B64 ? 3 : 2);
            if (B64) {
                const uint2 e = *reinterpret_cast<const uint2 *>(reinterpret_cast<const char *>(tab) + k * 256 + a);
                r = xor3(r, e.x, e.y);
            } else {
                r ^= *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(tab) + k * 128 + a);
            }
        }
        acc ^= r;
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    }
    if (acc == 0x12345678u)
        sink[0] = x;
}

#endif // ZDBCRC_DIAG

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void synth_kernel(uint8_t *__restrict__ buf, uint64_t len, uint64_t seed) {
    const uint64_t words = (len + 7) / 8;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < words;
         w += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t v = mix64(seed + (w + 1) * 0x9E3779B97F4A7C15ull);
        if (w * 8 + 8 <= len) {
            *reinterpret_cast<uint64_t *>(buf + w * 8) = v;
        } else {
            for (uint64_t k = 0; w * 8 + k < len; k++)
                buf[w * 8 + k] = (uint8_t)(v >> (8 * k));
        }
    }
}

// ---------------------------------------------------------------------------
// host side: per-device context, workspace, launch
// ---------------------------------------------------------------------------

struct Workspace {
    void *ptr = nullptr;
    size_t bytes = 0;
    uint32_t launches = 0; // checksum launches on this workspace (DYN counter parity)
};

struct DeviceCtx {
    bool ready = false;
    int cus = 0;
    uint32_t *d_tables = nullptr;
    std::map<void *, Workspace> ws; // per stream
};

// a launch bracketed by timing events (created on device `dev`)
struct TimedLaunch {
    int dev;
    hipEvent_t e0, e1;
    int kind; // 0: the main kernel; 1: the packed kernel of a split batch
};

// Locking: one mutex per device serialises that device's context,
// workspaces and host staging (calls on different devices -- one host thread
// per GPU in the multi-file scan -- run concurrently); g_mu guards the
// process-wide measurement state (pending timed launches, per-device event
// pools, accumulated time).
std::mutex g_mu;
std::mutex g_dev_mu[64];
DeviceCtx g_dev[64];
std::atomic<bool> g_hip_touched{false};
std::atomic<bool> g_timing{false};
std::vector<TimedLaunch> g_pending;
double g_time_ms[2] = {0, 0};
uint64_t g_launches[2] = {0, 0};
std::vector<hipEvent_t> g_event_pool[64]; // events are reused on the device they were created on
#ifdef ZDBCRC_DIAG
uint32_t *g_last_scratch = nullptr; // STAMP read-back (single-threaded measurement scripts)
#endif

std::vector<uint32_t> &host_tables() {
    static std::vector<uint32_t> t;
    static std::once_flag once;
    std::call_once(once, [] {
        t.resize(ZDBCRC_TABLE_DW);
        zdbcrc_build_tables(t.data());
    });
    return t;
}

// the calling thread's current HIP device (the device a call runs on)
int current_device(int *dev) {
    g_hip_touched = true;
    if (hipGetDevice(dev) != hipSuccess || *dev < 0 || *dev >= 64)
        return ZDB_CRC32_ENODEV;
    return ZDB_CRC32_OK;
}

// caller holds g_dev_mu[dev]
int ensure_device(int dev, DeviceCtx **out_ctx) {
    DeviceCtx &c = g_dev[dev];
    if (!c.ready) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) != hipSuccess)
            return ZDB_CRC32_ENODEV;
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            std::fprintf(stderr, "[-] zdbcrc: device %d is %s, this build targets gfx950\n", dev,
                         prop.gcnArchName);
            return ZDB_CRC32_ENODEV;
        }
        c.cus = prop.multiProcessorCount;
        std::vector<uint32_t> &t = host_tables();
        if (hipMalloc(&c.d_tables, t.size() * sizeof(uint32_t)) != hipSuccess)
            return ZDB_CRC32_ENOMEM;
        if (hipMemcpy(c.d_tables, t.data(), t.size() * sizeof(uint32_t), hipMemcpyHostToDevice) !=
            hipSuccess)
            return ZDB_CRC32_ELAUNCH;
        c.ready = true;
    }
    *out_ctx = &c;
    return ZDB_CRC32_OK;
}


// enqueue plan + main kernel; caller holds the device's g_dev_mu
// d_unit_start: the per-record unit prefix when the caller already has it
// (host-planned batches); nullptr -> computed on the device by the scan
// out_zeroed: a host-planned batch whose out[] is already zero (latency path)
int enqueue_batch(int dev, DeviceCtx &c, const KernelVariant &kv, const uint8_t *arena, const uint64_t *offsets,
                  const uint32_t *lengths, uint32_t *out, uint64_t n, hipStream_t st,
                  const uint64_t *d_unit_start = nullptr, uint32_t grid_wgs = 0, bool out_zeroed = false,
                  const uint64_t *d_n = nullptr) {
    if (n > 0xFFFFFFFFull) // record indices are 32-bit on the device (cut lists, mismatch indices)
        return ZDB_CRC32_EINVAL;
    // planner blocks: 2^lg records each (n + 1 entries), at most PLAN_MAX_BLOCKS
    uint32_t lg = 8; // one record per planner thread (PLAN_T = 256) until the block count limit
    while (((n + 1 + (1ull << lg) - 1) >> lg) > PLAN_MAX_BLOCKS)
        lg++;
    const uint64_t nb = (n + 1 + (1ull << lg) - 1) >> lg;
    // an unbounded, device-planned batch is split by record size (SPLIT_BYTES):
    // the packed kernel takes the small records, then kv the others
    const uint32_t split = d_unit_start ? 0u : split_bytes(kv);
    const int nplans = split ? 2 : 1;
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    const size_t local_bytes = d_unit_start ? 0 : al((n + 1) * sizeof(uint64_t));
    const size_t bsum_bytes = d_unit_start ? 0 : al(nb * sizeof(uint64_t));
    const size_t bmax_bytes = d_unit_start ? 0 : al(nb * sizeof(uint32_t));
    const size_t plan_bytes = local_bytes + bsum_bytes + bmax_bytes;
    // dummy dword per wave (64 KiB) | diagnostic stamps (448 KiB) | per-CU counters (4 KiB) | DYN counters (16 KiB)
    const size_t scratch_bytes = (64 + 448 + 4 + 16) * 1024;
    const size_t need = scratch_bytes + nplans * plan_bytes;
    Workspace &w = c.ws[reinterpret_cast<void *>(st)];
    if (w.bytes < need) {
        if (w.ptr) {
            hipDeviceSynchronize();
            hipFree(w.ptr);
            w.ptr = nullptr;
            w.bytes = 0;
        }
        if (hipMalloc(&w.ptr, need) != hipSuccess)
            return ZDB_CRC32_ENOMEM;
        w.bytes = need;
        if (hipMemsetAsync(w.ptr, 0, need, st) != hipSuccess)
            return ZDB_CRC32_ELAUNCH;
    }
    // scratch first: its offset must not move with n
    uint32_t *scratch = static_cast<uint32_t *>(w.ptr);
#ifdef ZDBCRC_DIAG
    g_last_scratch = scratch;
#endif
    PlanArgs plan{d_unit_start, nullptr, 0, 0, nullptr, d_n, 0};
    PlanArgs plan_s{};
    [[maybe_unused]] const KernelVariant &ks = split_variant(split ? split : 1);
    if (!d_unit_start) {
        PlanOut po[2];
        for (int k = 0; k < nplans; k++) {
            uint8_t *base = static_cast<uint8_t *>(w.ptr) + scratch_bytes + k * plan_bytes;
            po[k] = PlanOut{reinterpret_cast<uint64_t *>(base), reinterpret_cast<uint64_t *>(base + local_bytes),
                            reinterpret_cast<uint32_t *>(base + local_bytes + bsum_bytes)};
        }
#ifdef ZDBCRC_DIAG
        if (split)
            hipLaunchKernelGGL(plan_kernel<true>, dim3((uint32_t)nb), dim3(PLAN_T), 0, st, arena, offsets, lengths, n,
                               (uint64_t)kv.unit_ovh, lg, po[0], out, d_n, split, (uint64_t)ks.unit_ovh, po[1]);
        else
#endif
            hipLaunchKernelGGL(plan_kernel<false>, dim3((uint32_t)nb), dim3(PLAN_T), 0, st, arena, offsets, lengths,
                               n, (uint64_t)kv.unit_ovh, lg, po[0], out, d_n, 0u, (uint64_t)0, po[0]);
        if (hipGetLastError() != hipSuccess)
            return ZDB_CRC32_ELAUNCH;
        plan = PlanArgs{po[0].local, po[0].bsum, (uint32_t)nb, lg, po[0].bmax, d_n, 0};
        if (split)
            plan_s = PlanArgs{po[1].local, po[1].bsum, (uint32_t)nb, lg, po[1].bmax, d_n, split};
    } else if (!out_zeroed && hipMemsetAsync(out, 0, n * sizeof(uint32_t), st) != hipSuccess) {
        return ZDB_CRC32_ELAUNCH;
    }

    // full persistent grid, or fewer workgroups for a host-planned batch
    // that cannot occupy them (one SET value: the table fill of 512
    // workgroups would cost more than the checksum)
    uint32_t grid = (uint32_t)(c.cus * kv.wgs_per_cu);
    if (grid_wgs && grid_wgs < grid)
        grid = grid_wgs;
    const uint32_t max_waves = grid * (uint32_t)(kv.threads / 64);
    hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr, e3 = nullptr; // main kernel; packed kernel (split)
    std::unique_lock<std::mutex> tl(g_mu, std::defer_lock);
    if (g_timing.load()) {
        tl.lock();
        std::vector<hipEvent_t> &pool = g_event_pool[dev];
        // a pair of events, or none (no timing for a launch rather than a half-bracketed one)
        auto take = [&](hipEvent_t &a, hipEvent_t &b) {
            for (hipEvent_t *e : {&a, &b}) {
                if (!pool.empty()) {
                    *e = pool.back();
                    pool.pop_back();
                } else if (hipEventCreate(e) != hipSuccess) {
                    *e = nullptr;
                }
            }
            if (!a || !b) {
                for (hipEvent_t e : {a, b})
                    if (e)
                        pool.push_back(e);
                a = b = nullptr;
            }
        };
        take(e0, e1);
        if (split)
            take(e2, e3);
    }
    // the launch counter picks the tail-pool counter parity; it advances only
    // when a kernel was enqueued (each launch clears the next parity's counters)
    uint32_t ep = w.launches + 1;
    // timing: the dispatch packet itself carries the start/stop events
    // (hipExtLaunchKernel), so no marker packets sit between the kernels;
    // the packed kernel of a split batch has its own pair (kind 1)
#ifdef ZDBCRC_DIAG
    if (split) {
        const uint32_t sgrid = (uint32_t)(c.cus * ks.wgs_per_cu);
        const uint32_t swaves = sgrid * (uint32_t)(ks.threads / 64);
        if (e2)
            hipExtLaunchKernelGGL(ks.fn, dim3(sgrid), dim3(ks.threads), 0, st, e2, e3, 0u, arena, offsets,
                                  lengths, plan_s, n, out, c.d_tables, swaves, scratch, ep);
        else
            hipLaunchKernelGGL(ks.fn, dim3(sgrid), dim3(ks.threads), 0, st, arena, offsets, lengths, plan_s, n, out,
                               c.d_tables, swaves, scratch, ep);
        if (hipGetLastError() != hipSuccess)
            return ZDB_CRC32_ELAUNCH;
        w.launches = ep++;
    }
#endif
    if (e0)
        hipExtLaunchKernelGGL(kv.fn, dim3(grid), dim3(kv.threads), 0, st, e0, e1, 0u, arena, offsets, lengths,
                              plan, n, out, c.d_tables, max_waves, scratch, ep);
    else
        hipLaunchKernelGGL(kv.fn, dim3(grid), dim3(kv.threads), 0, st, arena, offsets, lengths, plan, n,
                           out, c.d_tables, max_waves, scratch, ep);
    if (hipGetLastError() != hipSuccess)
        return ZDB_CRC32_ELAUNCH;
    w.launches = ep;
    if (e1)
        g_pending.push_back(TimedLaunch{dev, e0, e1, 0});
    if (e3)
        g_pending.push_back(TimedLaunch{dev, e2, e3, 1});
    return ZDB_CRC32_OK;
}

struct HostStaging {
    uint8_t *arena = nullptr; // device copy of the caller's arena
    size_t arena_bytes = 0;
    uint8_t *plan = nullptr;  // device: offsets | lengths | unit_start | out
    uint8_t *hplan = nullptr; // pinned host mirror of plan
    size_t n_cap = 0;
    uint32_t *mbox = nullptr; // mapped host-coherent: seq word, pad, MAILBOX_RECORDS results
    uint32_t *d_mbox = nullptr;
    uint32_t *d_mout = nullptr; // device results of the latency path, MAILBOX_RECORDS
    bool mout_zeroed = false;   // all of d_mout is zero (publish_kernel re-zeroes what a batch used)
    uint32_t seq = 0;
    hipStream_t st = nullptr;
};

// wait for publish_kernel's sequence word; a failed or faulted stream ends
// the wait through hipStreamQuery, a long batch through a blocking sync
int wait_mailbox(HostStaging &h, uint32_t seq) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spins = 1;; spins++) {
        if (__atomic_load_n(h.mbox, __ATOMIC_ACQUIRE) == seq)
            return ZDB_CRC32_OK;
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
        if ((spins & 255) != 0)
            continue;
        const hipError_t q = hipStreamQuery(h.st);
        if (q != hipSuccess && q != hipErrorNotReady)
            return ZDB_CRC32_ELAUNCH;
        if (q == hipErrorNotReady && std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(500))
            continue;
        if (q == hipErrorNotReady && hipStreamSynchronize(h.st) != hipSuccess)
            return ZDB_CRC32_ELAUNCH;
        // the stream has drained: the word is there, or the batch failed
        return __atomic_load_n(h.mbox, __ATOMIC_ACQUIRE) == seq ? ZDB_CRC32_OK : ZDB_CRC32_ELAUNCH;
    }
}
HostStaging g_host_staging[64];

// pinned allocations made by zdb_crc32_host_alloc (base -> bytes, including
// 64 readable bytes past what the caller asked for) and ranges pinned by
// zdb_crc32_host_register (base -> bytes): a host-buffer batch
// whose arena lies inside one is read by the kernel in place, over PCIe
// (zero-copy), with no staging copy
std::mutex g_pin_mu;
std::map<uintptr_t, size_t> g_pinned;

const uint8_t *pinned_device_view(const uint8_t *arena, size_t len) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(arena);
    std::lock_guard<std::mutex> g(g_pin_mu);
    auto it = g_pinned.upper_bound(a);
    if (it == g_pinned.begin())
        return nullptr;
    --it;
    if (a + len + 16 > it->first + it->second) // the kernel reads up to the next 16-byte boundary
        return nullptr;
    void *dp = nullptr;
    if (hipHostGetDevicePointer(&dp, reinterpret_cast<void *>(it->first), 0) != hipSuccess || !dp)
        return nullptr;
    return static_cast<const uint8_t *>(dp) + (a - it->first);
}

// [p, p + n) inside one pinned range (allocated or registered)
bool pinned_range(const uint8_t *p, size_t n) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::lock_guard<std::mutex> g(g_pin_mu);
    auto it = g_pinned.upper_bound(a);
    if (it == g_pinned.begin())
        return false;
    --it;
    return a + n <= it->first + it->second;
}

size_t plan_bytes(size_t n) { return n * 8 + n * 4 + (n + 1) * 8 + n * 4 + 64; }

} // namespace

extern "C" {

const char *zdb_crc32_strerror(int code) {
    switch (code) {
    case ZDB_CRC32_OK: return "ok";
    case ZDB_CRC32_ENODEV: return "no usable gfx950 HIP device";
    case ZDB_CRC32_EINVAL: return "invalid argument";
    case ZDB_CRC32_ENOMEM: return "device allocation failed";
    case ZDB_CRC32_ELAUNCH: return "HIP launch/runtime error";
    case ZDB_CRC32_ENOSPC: return "output buffers too small";
    default: return "unknown error";
    }
}

// the engine of the calling thread's current device; never initialises HIP
const char *zdb_crc32_batch_engine(void) {
    if (!g_hip_touched.load())
        return "uninitialized";
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64)
        return "uninitialized";
    std::lock_guard<std::mutex> g(g_dev_mu[dev]);
    return g_dev[dev].ready ? "hip-gfx950" : "uninitialized";
}

int zdb_crc32_gpu_initialized(void) { return g_hip_touched ? 1 : 0; }

// library-internal (not in the version script): other HIP objects of
// libzdbcrc.so record that they initialised HIP
void zdbcrc_internal_mark_hip(void) { g_hip_touched = true; }

#ifdef ZDBCRC_DIAG
// measurement hook (not part of the public ABI): time a read-only stream of
// `bytes` (multiple of 16) with HIP events; returns ms, <0 on error
float zdbcrc_debug_stream_read(const void *d_buf, size_t bytes, uint32_t *d_sink, int blocks, void *stream) {
    hipStream_t st = static_cast<hipStream_t>(stream);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, st);
    const uint4 *src = static_cast<const uint4 *>(d_buf);
    const uint64_t words = bytes / 16;
    // blocks > 0: grid-stride probe with that many 256-thread blocks;
    // blocks = -U: contiguous-slice probe, 512 x 1024-thread blocks, U loads/lane
    // blocks = -100 - U: the same with nontemporal loads
    if (blocks > 0)
        hipLaunchKernelGGL(stream_read_kernel, dim3(blocks), dim3(256), 0, st, src, words, d_sink);
    else if (blocks == -4)
        hipLaunchKernelGGL(stream_slice_kernel<4>, dim3(512), dim3(1024), 0, st, src, words, d_sink);
    else if (blocks == -8)
        hipLaunchKernelGGL(stream_slice_kernel<8>, dim3(512), dim3(1024), 0, st, src, words, d_sink);
    else if (blocks == -104)
        hipLaunchKernelGGL((stream_slice_kernel<4, true>), dim3(512), dim3(1024), 0, st, src, words, d_sink);
    else if (blocks == -204)
        hipLaunchKernelGGL((stream_slice_kernel<4, true>), dim3(512), dim3(768), 0, st, src, words, d_sink);
    else if (blocks == -202) // 768 threads, 2 / 1 loads in flight per lane (bytes in flight per CU: 48 / 24 KiB)
        hipLaunchKernelGGL((stream_slice_kernel<2, true>), dim3(512), dim3(768), 0, st, src, words, d_sink);
    else if (blocks == -201)
        hipLaunchKernelGGL((stream_slice_kernel<1, true>), dim3(512), dim3(768), 0, st, src, words, d_sink);
    else if (blocks == -208)
        hipLaunchKernelGGL((stream_slice_kernel<8, true>), dim3(512), dim3(768), 0, st, src, words, d_sink);
    else if (blocks == -108)
        hipLaunchKernelGGL((stream_slice_kernel<8, true>), dim3(512), dim3(1024), 0, st, src, words, d_sink);
    else if (blocks == -304) // packed access shapes (stream_rows_kernel): rows of 4 / 8 / 16 / 64 lanes
        hipLaunchKernelGGL((stream_rows_kernel<4, 4>), dim3(512), dim3(1024), 0, st, src, words, d_sink);
    else if (blocks == -308)
        hipLaunchKernelGGL((stream_rows_kernel<8, 4>), dim3(512), dim3(1024), 0, st, src, words, d_sink);
    else if (blocks == -316)
        hipLaunchKernelGGL((stream_rows_kernel<16, 4>), dim3(512), dim3(1024), 0, st, src, words, d_sink);
    else if (blocks == -364)
        hipLaunchKernelGGL((stream_rows_kernel<64, 4>), dim3(512), dim3(1024), 0, st, src, words, d_sink);
    else if (blocks == -344) // rows of 4 lanes, 8 loads in flight
        hipLaunchKernelGGL((stream_rows_kernel<4, 8>), dim3(512), dim3(1024), 0, st, src, words, d_sink);
    else
        hipLaunchKernelGGL(stream_slice_kernel<16>, dim3(512), dim3(1024), 0, st, src, words, d_sink);
    hipEventRecord(b, st);
    float ms = -1;
    if (hipEventSynchronize(b) == hipSuccess)
        hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ms;
}

// measurement hook: LDS lookup microbenchmark, mode 0..3 = (V 1|2) x (b32|b64);
// returns ms for one launch of 2 x 768-thread workgroups per CU
float zdbcrc_debug_lds_bench(int mode, uint32_t iters, uint32_t *d_sink, int cus, void *stream) {
    hipStream_t st = static_cast<hipStream_t>(stream);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, st);
    const dim3 grid(2 * cus), blk(768);
    switch (mode) {
    case 0: hipLaunchKernelGGL((lds_bench_kernel<1, false>), grid, blk, 0, st, iters, d_sink); break;
    case 1: hipLaunchKernelGGL((lds_bench_kernel<2, false>), grid, blk, 0, st, iters, d_sink); break;
    case 2: hipLaunchKernelGGL((lds_bench_kernel<1, true>), grid, blk, 0, st, iters, d_sink); break;
    default: hipLaunchKernelGGL((lds_bench_kernel<2, true>), grid, blk, 0, st, iters, d_sink); break;
    }
    hipEventRecord(b, st);
    float ms = -1;
    if (hipEventSynchronize(b) == hipSuccess)
        hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ms;
}

// measurement hook: copy the per-wave (start, end) stamps of the last launch
// of a STAMP variant (waves * 2 u64) to host memory
int zdbcrc_debug_read_stamps(uint64_t *host, size_t waves) {
    if (!g_last_scratch || waves > 8192)
        return -1;
    return hipMemcpy(host, g_last_scratch + 16384, waves * 32, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}

// measurement hook (not part of the public ABI): select a kernel variant for
// A/B timing in one process; returns its name, NULL if out of range
// A/B: split unbounded batches at this many bytes (0: never)
int zdbcrc_debug_set_split(uint32_t bytes) {
    g_debug_split.store(bytes);
    return 0;
}

const char *zdbcrc_debug_set_variant(int idx) {
    if (idx < 0 || idx >= kNumVariants)
        return nullptr;
    g_variant = idx;
    return kVariants[idx].name;
}

// measurement hook: how a small host batch returns its results (0 the
// mailbox, as shipped; 1 device memset + copy + stream sync)
int zdbcrc_debug_set_host_mode(int mode) {
    if (mode < 0 || mode > 1)
        return -1;
    g_host_mode = mode;
    return 0;
}

#endif // ZDBCRC_DIAG

int zdb_crc32_batch_device(const uint8_t *d_arena, const uint64_t *d_offsets, const uint32_t *d_lengths,
                           uint32_t *d_out, size_t n, void *stream) {
    if (n == 0)
        return ZDB_CRC32_OK;
    if (!d_arena || !d_offsets || !d_lengths || !d_out)
        return ZDB_CRC32_EINVAL;
    int dev;
    int rc = current_device(&dev);
    if (rc)
        return rc;
    std::lock_guard<std::mutex> g(g_dev_mu[dev]);
    DeviceCtx *c;
    if ((rc = ensure_device(dev, &c)))
        return rc;
    return enqueue_batch(dev, *c, variant(), d_arena, d_offsets, d_lengths, d_out, n,
                         static_cast<hipStream_t>(stream));
}

int zdb_crc32_batch_device_sized(const uint8_t *d_arena, const uint64_t *d_offsets, const uint32_t *d_lengths,
                                 uint32_t *d_out, size_t n, uint32_t max_length, void *stream) {
    if (n == 0)
        return ZDB_CRC32_OK;
    if (!d_arena || !d_offsets || !d_lengths || !d_out)
        return ZDB_CRC32_EINVAL;
    int dev;
    int rc = current_device(&dev);
    if (rc)
        return rc;
    std::lock_guard<std::mutex> g(g_dev_mu[dev]);
    DeviceCtx *c;
    if ((rc = ensure_device(dev, &c)))
        return rc;
    return enqueue_batch(dev, *c, variant(max_length), d_arena, d_offsets, d_lengths, d_out, n,
                         static_cast<hipStream_t>(stream));
}

// zdb_crc32_verify_device with, optionally, the record count in device
// memory (d_n; n is then its bound): the f3 scan verifies what its walk
// found without a host round trip for the count (not exported)
int zdbcrc_internal_verify_device_dn(const uint8_t *d_arena, const uint64_t *d_offsets, const uint32_t *d_lengths,
                                     const uint32_t *d_expected, uint32_t *d_out, uint32_t *d_mismatch,
                                     uint32_t *d_mismatch_count, uint32_t max_mismatch, size_t n,
                                     const uint64_t *d_n, void *stream) {
    if (!d_mismatch_count || !d_expected || (max_mismatch && !d_mismatch))
        return ZDB_CRC32_EINVAL;
    hipStream_t st = static_cast<hipStream_t>(stream);
    {
        int dev;
        int rc = current_device(&dev);
        if (rc)
            return rc;
        std::lock_guard<std::mutex> g(g_dev_mu[dev]);
        DeviceCtx *c;
        if ((rc = ensure_device(dev, &c)))
            return rc;
        if (hipMemsetAsync(d_mismatch_count, 0, sizeof(uint32_t), st) != hipSuccess)
            return ZDB_CRC32_ELAUNCH;
        if (n == 0)
            return ZDB_CRC32_OK;
        if (!d_arena || !d_offsets || !d_lengths || !d_out)
            return ZDB_CRC32_EINVAL;
        rc = enqueue_batch(dev, *c, variant(), d_arena, d_offsets, d_lengths, d_out, n, st, nullptr, 0, false, d_n);
        if (rc)
            return rc;
    }
    const uint32_t blocks = (uint32_t)((n + 255) / 256);
    hipLaunchKernelGGL(verify_kernel, dim3(blocks), dim3(256), 0, st, d_out, d_expected, (uint64_t)n,
                       d_mismatch, d_mismatch_count, max_mismatch, d_n);
    return hipGetLastError() == hipSuccess ? ZDB_CRC32_OK : ZDB_CRC32_ELAUNCH;
}

int zdb_crc32_verify_device(const uint8_t *d_arena, const uint64_t *d_offsets, const uint32_t *d_lengths,
                            const uint32_t *d_expected, uint32_t *d_out, uint32_t *d_mismatch,
                            uint32_t *d_mismatch_count, uint32_t max_mismatch, size_t n, void *stream) {
    return zdbcrc_internal_verify_device_dn(d_arena, d_offsets, d_lengths, d_expected, d_out, d_mismatch,
                                            d_mismatch_count, max_mismatch, n, nullptr, stream);
}

int zdb_datafile_check_device(const uint8_t *d_image, uint64_t image_len, const uint64_t *d_offsets,
                              int32_t *d_result, size_t n, void *stream) {
    if (n == 0)
        return ZDB_CRC32_OK;
    if (!d_image || !d_offsets || !d_result)
        return ZDB_CRC32_EINVAL;
    hipStream_t st = static_cast<hipStream_t>(stream);
    int dev;
    int rc = current_device(&dev);
    if (rc)
        return rc;
    std::lock_guard<std::mutex> g(g_dev_mu[dev]);
    DeviceCtx *c;
    if ((rc = ensure_device(dev, &c)))
        return rc;
    // descriptors: offsets (8 B) | lengths, expected, out (4 B each) per record
    void *tmp = nullptr;
    if (hipMallocAsync(&tmp, n * 20, st) != hipSuccess)
        return ZDB_CRC32_ENOMEM;
    uint64_t *offs = static_cast<uint64_t *>(tmp);
    uint32_t *lens = reinterpret_cast<uint32_t *>(offs + n);
    uint32_t *expect = lens + n;
    uint32_t *out = expect + n;
    const uint32_t blocks = (uint32_t)((n + 255) / 256);
    hipLaunchKernelGGL(check_decode_kernel, dim3(blocks), dim3(256), 0, st, d_image, image_len, d_offsets,
                       (uint64_t)n, offs, lens, expect, d_result);
    rc = hipGetLastError() == hipSuccess ? ZDB_CRC32_OK : ZDB_CRC32_ELAUNCH;
    if (!rc)
        rc = enqueue_batch(dev, *c, variant(), d_image, offs, lens, out, n, st);
    if (!rc) {
        hipLaunchKernelGGL(check_finish_kernel, dim3(blocks), dim3(256), 0, st, out, expect, (uint64_t)n,
                           d_result);
        rc = hipGetLastError() == hipSuccess ? ZDB_CRC32_OK : ZDB_CRC32_ELAUNCH;
    }
    hipFreeAsync(tmp, st);
    return rc;
}

int zdb_crc32_batch(const uint8_t *arena, size_t arena_len, const uint64_t *offsets, const uint32_t *lengths,
                    uint32_t *out, size_t n) {
    if (n == 0)
        return ZDB_CRC32_OK;
    if (!arena || !offsets || !lengths || !out)
        return ZDB_CRC32_EINVAL;
    uint32_t max_len = 0;
    for (size_t r = 0; r < n; r++) { // overflow-safe: offsets[r] may be near UINT64_MAX
        if (offsets[r] > arena_len || lengths[r] > arena_len - offsets[r])
            return ZDB_CRC32_EINVAL;
        max_len = lengths[r] > max_len ? lengths[r] : max_len;
    }
    int dev;
    int rc = current_device(&dev);
    if (rc)
        return rc;
    std::lock_guard<std::mutex> g(g_dev_mu[dev]);
    DeviceCtx *c;
    if ((rc = ensure_device(dev, &c)))
        return rc;
    HostStaging &h = g_host_staging[dev];
    if (!h.st && hipStreamCreateWithFlags(&h.st, hipStreamNonBlocking) != hipSuccess)
        return ZDB_CRC32_ELAUNCH;
    // an arena in memory from zdb_crc32_host_alloc is read in place (C5:
    // one SET value costs a launch and a sync instead of two copies more)
    const uint8_t *d_arena = pinned_device_view(arena, arena_len);
    const size_t abytes = arena_len + 16;
    if (!d_arena && h.arena_bytes < abytes) {
        if (h.arena)
            hipFree(h.arena);
        h.arena = nullptr;
        if (hipMalloc(&h.arena, abytes) != hipSuccess) {
            h.arena_bytes = 0;
            return ZDB_CRC32_ENOMEM;
        }
        h.arena_bytes = abytes;
    }
    if (h.n_cap < n) {
        if (h.plan)
            hipFree(h.plan);
        if (h.hplan)
            hipHostFree(h.hplan);
        h.plan = nullptr;
        h.hplan = nullptr;
        if (hipMalloc(&h.plan, plan_bytes(n)) != hipSuccess ||
            hipHostMalloc(&h.hplan, plan_bytes(n), hipHostMallocDefault) != hipSuccess) {
            h.n_cap = 0;
            return ZDB_CRC32_ENOMEM;
        }
        h.n_cap = n;
    }
    if (n <= MAILBOX_RECORDS && !h.mbox) {
        void *m = nullptr, *dm = nullptr;
        if (!h.d_mout && hipMalloc(&h.d_mout, MAILBOX_RECORDS * 4) != hipSuccess) {
            h.d_mout = nullptr;
            return ZDB_CRC32_ENOMEM;
        }
        if (hipHostMalloc(&m, (MAILBOX_PAD + MAILBOX_RECORDS) * 4, hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess)
            return ZDB_CRC32_ENOMEM;
        if (hipHostGetDevicePointer(&dm, m, 0) != hipSuccess || !dm) {
            hipHostFree(m);
            return ZDB_CRC32_ELAUNCH;
        }
        std::memset(m, 0, (MAILBOX_PAD + MAILBOX_RECORDS) * 4);
        h.mbox = static_cast<uint32_t *>(m);
        h.d_mbox = static_cast<uint32_t *>(dm);
    }
    // host-side planning: the descriptors and the unit prefix go over in one
    // copy, so a small batch (one SET value) needs no device scan
    uint64_t *ho = reinterpret_cast<uint64_t *>(h.hplan);
    uint32_t *hl = reinterpret_cast<uint32_t *>(h.hplan + n * 8);
    uint64_t *hu = reinterpret_cast<uint64_t *>(h.hplan + n * 12);
    uint32_t *hout = reinterpret_cast<uint32_t *>(h.hplan + n * 12 + (n + 1) * 8);
    std::memcpy(ho, offsets, n * 8);
    std::memcpy(hl, lengths, n * 4);
    // resolved once: the host prefix and the kernel agree on UO
#ifdef ZDBCRC_DIAG
    const bool mailbox = n <= MAILBOX_RECORDS && g_host_mode.load() == 0; // A/B: 1 = copy + sync
#else
    const bool mailbox = n <= MAILBOX_RECORDS;
#endif
    const KernelVariant &kv = variant(max_len ? max_len : 1); // all empty: any shape
    if (!d_arena)
        d_arena = h.arena;
    const UnitCount uc{d_arena, offsets, lengths, n, kv.unit_ovh};
    uint64_t acc = 0;
    for (size_t r = 0; r < n; r++) {
        hu[r] = acc;
        acc += uc(r);
    }
    hu[n] = acc;
    uint64_t *d_off = reinterpret_cast<uint64_t *>(h.plan);
    uint32_t *d_len = reinterpret_cast<uint32_t *>(h.plan + n * 8);
    uint64_t *d_us = reinterpret_cast<uint64_t *>(h.plan + n * 12);
    uint32_t *d_out = reinterpret_cast<uint32_t *>(h.plan + n * 12 + (n + 1) * 8);
    const bool zero_copy = d_arena != h.arena;
    if (zero_copy) { // the descriptors too are read in place from the pinned plan
        void *dp = nullptr;
        if (hipHostGetDevicePointer(&dp, h.hplan, 0) != hipSuccess || !dp)
            return ZDB_CRC32_ELAUNCH;
        uint8_t *dplan = static_cast<uint8_t *>(dp);
        d_off = reinterpret_cast<uint64_t *>(dplan);
        d_len = reinterpret_cast<uint32_t *>(dplan + n * 8);
        d_us = reinterpret_cast<uint64_t *>(dplan + n * 12);
    } else if (hipMemcpyAsync(h.arena, arena, arena_len, hipMemcpyHostToDevice, h.st) != hipSuccess ||
               hipMemcpyAsync(h.plan, h.hplan, n * 12 + (n + 1) * 8, hipMemcpyHostToDevice, h.st) != hipSuccess) {
        return ZDB_CRC32_ELAUNCH;
    }
    // workgroups the batch can keep busy (MIN_UNITS_PER_WAVE units per wave)
    const uint64_t waves = (acc + MIN_UNITS_PER_WAVE - 1) / MIN_UNITS_PER_WAVE;
    const uint64_t wpw = (uint64_t)(kv.threads / 64);
    const uint32_t grid_wgs = (uint32_t)std::min<uint64_t>((waves + wpw - 1) / wpw, 1u << 20);
    if (mailbox) {
        if (!h.mout_zeroed && hipMemsetAsync(h.d_mout, 0, MAILBOX_RECORDS * 4, h.st) != hipSuccess)
            return ZDB_CRC32_ELAUNCH;
        d_out = h.d_mout;
        h.mout_zeroed = false; // until the batch has published
    }
    const uint32_t seq = mailbox ? (++h.seq ? h.seq : ++h.seq) : 0; // never 0, the mailbox's initial value
    rc = enqueue_batch(dev, *c, kv, d_arena, d_off, d_len, d_out, n, h.st, d_us, grid_wgs, mailbox);
    if (rc)
        return rc;
    if (mailbox) { // C5 latency path: results through the mailbox
        hipLaunchKernelGGL(publish_kernel, dim3(1), dim3(64), 0, h.st, d_out, h.d_mbox + MAILBOX_PAD, (uint32_t)n,
                           h.d_mbox, seq);
        if (hipGetLastError() != hipSuccess)
            return ZDB_CRC32_ELAUNCH;
        if ((rc = wait_mailbox(h, seq)))
            return rc;
        h.mout_zeroed = true;
        std::memcpy(out, h.mbox + MAILBOX_PAD, n * 4);
        return ZDB_CRC32_OK;
    }
    if (hipMemcpyAsync(hout, d_out, n * 4, hipMemcpyDeviceToHost, h.st) != hipSuccess)
        return ZDB_CRC32_ELAUNCH;
    if (hipStreamSynchronize(h.st) != hipSuccess)
        return ZDB_CRC32_ELAUNCH;
    std::memcpy(out, hout, n * 4);
    return ZDB_CRC32_OK;
}

int zdb_crc32_device_count(void) {
    g_hip_touched = true;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess)
        return 0;
    return n;
}

int zdb_crc32_use_device(int device) {
    g_hip_touched = true;
    if (device < 0 || device >= 64)
        return ZDB_CRC32_EINVAL;
    return hipSetDevice(device) == hipSuccess ? ZDB_CRC32_OK : ZDB_CRC32_ENODEV;
}

void *zdb_crc32_host_alloc(size_t bytes) {
    g_hip_touched = true;
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes + 64, hipHostMallocDefault) != hipSuccess)
        return nullptr;
    std::lock_guard<std::mutex> g(g_pin_mu);
    g_pinned[reinterpret_cast<uintptr_t>(p)] = bytes + 64;
    return p;
}

void zdb_crc32_host_free(void *p) {
    if (!p)
        return;
    {
        std::lock_guard<std::mutex> g(g_pin_mu);
        g_pinned.erase(reinterpret_cast<uintptr_t>(p));
    }
    hipHostFree(p);
}

int zdb_crc32_host_register(void *p, size_t bytes) {
    g_hip_touched = true;
    if (!p || !bytes)
        return ZDB_CRC32_EINVAL;
    if (hipHostRegister(p, bytes, hipHostRegisterPortable | hipHostRegisterMapped) != hipSuccess)
        return ZDB_CRC32_ENOMEM;
    std::lock_guard<std::mutex> g(g_pin_mu);
    g_pinned[reinterpret_cast<uintptr_t>(p)] = bytes;
    return ZDB_CRC32_OK;
}

void zdb_crc32_host_unregister(void *p) {
    if (!p)
        return;
    {
        std::lock_guard<std::mutex> g(g_pin_mu);
        g_pinned.erase(reinterpret_cast<uintptr_t>(p));
    }
    hipHostUnregister(p);
}

void zdb_crc32_set_timing(int enable) {
    std::lock_guard<std::mutex> g(g_mu);
    g_timing.store(enable != 0);
}

static int drain_timing(float *each, size_t max_each, size_t *n_each) {
    size_t k = 0;
    for (const TimedLaunch &p : g_pending) {
        if (hipEventSynchronize(p.e1) != hipSuccess)
            return ZDB_CRC32_ELAUNCH;
        float ms = 0;
        hipEventElapsedTime(&ms, p.e0, p.e1);
        g_time_ms[p.kind] += ms;
        g_launches[p.kind] += 1;
        if (each && k < max_each && p.kind == 0)
            each[k++] = ms;
        g_event_pool[p.dev].push_back(p.e0);
        g_event_pool[p.dev].push_back(p.e1);
    }
    g_pending.clear();
    if (n_each)
        *n_each = k;
    return ZDB_CRC32_OK;
}

#ifdef ZDBCRC_DIAG
// debug: per-launch kernel times (ms) recorded since the last drain
long zdbcrc_debug_kernel_times(float *each, size_t max_each) {
    std::lock_guard<std::mutex> g(g_mu);
    size_t k = 0;
    if (drain_timing(each, max_each, &k))
        return -1;
    g_time_ms[0] = g_time_ms[1] = 0;
    g_launches[0] = g_launches[1] = 0;
    return (long)k;
}

#endif // ZDBCRC_DIAG

static int kernel_stats_of(int kind, double *total_ms, uint64_t *launches) {
    std::lock_guard<std::mutex> g(g_mu);
    if (int rc = drain_timing(nullptr, 0, nullptr))
        return rc;
    if (total_ms)
        *total_ms = g_time_ms[kind];
    if (launches)
        *launches = g_launches[kind];
    g_time_ms[kind] = 0;
    g_launches[kind] = 0;
    return ZDB_CRC32_OK;
}

int zdb_crc32_kernel_stats(double *total_ms, uint64_t *launches) { return kernel_stats_of(0, total_ms, launches); }

#ifdef ZDBCRC_DIAG
// debug: the packed kernel of split batches (A/B of zdbcrc_debug_set_split)
int zdbcrc_debug_small_kernel_stats(double *total_ms, uint64_t *launches) {
    return kernel_stats_of(1, total_ms, launches);
}
#endif

// ---------------------------------------------------------------------------
// f1: host -> device ingest stream (include/zdb_crc32.h, section 2b)
// ---------------------------------------------------------------------------

struct zdb_crc32_stream_t {
    int dev = -1;
    hipStream_t st = nullptr;
    uint8_t *d_image = nullptr; // device image of the current file
    size_t d_cap = 0, cap = 0, fill = 0;
    size_t slot_bytes = 0;
    int nslots = 0, next = 0;
    uint8_t *slot[ZDB_CRC32_STREAM_MAX_SLOTS] = {};
    hipEvent_t done[ZDB_CRC32_STREAM_MAX_SLOTS] = {};
    bool used[ZDB_CRC32_STREAM_MAX_SLOTS] = {};
    uint8_t *d_desc = nullptr, *h_desc = nullptr; // offsets (8 n) | lengths (4 n) | out (4 n)
    size_t desc_cap = 0;
};

static void stream_free(zdb_crc32_stream_t *s) {
    if (!s)
        return;
    if (s->dev >= 0)
        hipSetDevice(s->dev);
    if (s->st)
        hipStreamSynchronize(s->st);
    for (int i = 0; i < s->nslots; i++) {
        if (s->slot[i])
            hipHostFree(s->slot[i]);
        if (s->done[i])
            hipEventDestroy(s->done[i]);
    }
    if (s->d_image)
        hipFree(s->d_image);
    if (s->d_desc)
        hipFree(s->d_desc);
    if (s->h_desc)
        hipHostFree(s->h_desc);
    if (s->st) {
        std::lock_guard<std::mutex> g(g_dev_mu[s->dev]);
        auto it = g_dev[s->dev].ws.find(reinterpret_cast<void *>(s->st));
        if (it != g_dev[s->dev].ws.end()) {
            hipFree(it->second.ptr);
            g_dev[s->dev].ws.erase(it);
        }
        hipStreamDestroy(s->st);
    }
    delete s;
}

zdb_crc32_stream_t *zdb_crc32_stream_open(size_t slot_bytes, int slots) {
    if (slot_bytes < 4096 || slots < 2 || slots > ZDB_CRC32_STREAM_MAX_SLOTS)
        return nullptr;
    int dev;
    if (current_device(&dev))
        return nullptr;
    {
        std::lock_guard<std::mutex> g(g_dev_mu[dev]);
        DeviceCtx *c;
        if (ensure_device(dev, &c))
            return nullptr;
    }
    zdb_crc32_stream_t *s = new zdb_crc32_stream_t;
    s->dev = dev;
    s->slot_bytes = slot_bytes;
    s->nslots = slots;
    bool ok = hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking) == hipSuccess;
    for (int i = 0; ok && i < slots; i++)
        ok = hipHostMalloc(reinterpret_cast<void **>(&s->slot[i]), slot_bytes, hipHostMallocDefault) == hipSuccess &&
             hipEventCreateWithFlags(&s->done[i], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        stream_free(s);
        return nullptr;
    }
    return s;
}

int zdb_crc32_stream_begin(zdb_crc32_stream_t *s, size_t image_bytes) {
    if (!s)
        return ZDB_CRC32_EINVAL;
    if (hipSetDevice(s->dev) != hipSuccess || hipStreamSynchronize(s->st) != hipSuccess)
        return ZDB_CRC32_ELAUNCH;
    const size_t need = image_bytes + 16; // the kernel may read up to the next 16-byte boundary
    if (s->d_cap < need) {
        if (s->d_image)
            hipFree(s->d_image);
        s->d_image = nullptr;
        s->d_cap = 0;
        const size_t cap = need + (need >> 3);
        if (hipMalloc(reinterpret_cast<void **>(&s->d_image), cap) != hipSuccess)
            return ZDB_CRC32_ENOMEM;
        s->d_cap = cap;
    }
    s->cap = image_bytes;
    s->fill = 0;
    return ZDB_CRC32_OK;
}

int zdb_crc32_stream_append(zdb_crc32_stream_t *s, const uint8_t *src, size_t n) {
    if (!s || (n && !src) || n > s->cap - s->fill)
        return ZDB_CRC32_EINVAL;
    if (hipSetDevice(s->dev) != hipSuccess)
        return ZDB_CRC32_ELAUNCH;
    if (n && pinned_range(src, n)) {
        // pinned source (zdb_crc32_host_alloc / _register): one DMA straight
        // from it, no staging copy and no wait -- the caller keeps the bytes
        // until the next begin or checksum, which wait for the copy
        if (hipMemcpyAsync(s->d_image + s->fill, src, n, hipMemcpyHostToDevice, s->st) != hipSuccess)
            return ZDB_CRC32_ELAUNCH;
        s->fill += n;
        return ZDB_CRC32_OK;
    }
    while (n) {
        const int i = s->next;
        // the slot is free again once its previous copy has left it
        if (s->used[i] && hipEventSynchronize(s->done[i]) != hipSuccess)
            return ZDB_CRC32_ELAUNCH;
        const size_t k = n < s->slot_bytes ? n : s->slot_bytes;
        std::memcpy(s->slot[i], src, k);
        if (hipMemcpyAsync(s->d_image + s->fill, s->slot[i], k, hipMemcpyHostToDevice, s->st) != hipSuccess ||
            hipEventRecord(s->done[i], s->st) != hipSuccess)
            return ZDB_CRC32_ELAUNCH;
        s->used[i] = true;
        s->fill += k;
        src += k;
        n -= k;
        s->next = (i + 1) % s->nslots;
    }
    return ZDB_CRC32_OK;
}

int zdb_crc32_stream_checksum(zdb_crc32_stream_t *s, const uint64_t *offsets, const uint32_t *lengths,
                              uint32_t *out, size_t n) {
    if (!s)
        return ZDB_CRC32_EINVAL;
    if (n == 0)
        return ZDB_CRC32_OK;
    if (!offsets || !lengths || !out)
        return ZDB_CRC32_EINVAL;
    uint32_t max_len = 0;
    for (size_t r = 0; r < n; r++) { // overflow-safe bounds against the appended bytes
        if (offsets[r] > s->fill || lengths[r] > s->fill - offsets[r])
            return ZDB_CRC32_EINVAL;
        max_len = lengths[r] > max_len ? lengths[r] : max_len;
    }
    if (hipSetDevice(s->dev) != hipSuccess)
        return ZDB_CRC32_ELAUNCH;
    const size_t need = n * 16 + 64;
    if (s->desc_cap < need) {
        if (hipStreamSynchronize(s->st) != hipSuccess)
            return ZDB_CRC32_ELAUNCH;
        if (s->d_desc)
            hipFree(s->d_desc);
        if (s->h_desc)
            hipHostFree(s->h_desc);
        s->d_desc = s->h_desc = nullptr;
        s->desc_cap = 0;
        const size_t cap = need + (need >> 2);
        if (hipMalloc(reinterpret_cast<void **>(&s->d_desc), cap) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void **>(&s->h_desc), cap, hipHostMallocDefault) != hipSuccess)
            return ZDB_CRC32_ENOMEM;
        s->desc_cap = cap;
    }
    std::memcpy(s->h_desc, offsets, n * 8);
    std::memcpy(s->h_desc + n * 8, lengths, n * 4);
    if (hipMemcpyAsync(s->d_desc, s->h_desc, n * 12, hipMemcpyHostToDevice, s->st) != hipSuccess)
        return ZDB_CRC32_ELAUNCH;
    uint32_t *d_out = reinterpret_cast<uint32_t *>(s->d_desc + n * 12);
    {
        std::lock_guard<std::mutex> g(g_dev_mu[s->dev]);
        DeviceCtx *c;
        int rc = ensure_device(s->dev, &c);
        if (!rc)
            rc = enqueue_batch(s->dev, *c, variant(max_len ? max_len : 1), s->d_image,
                               reinterpret_cast<const uint64_t *>(s->d_desc),
                               reinterpret_cast<const uint32_t *>(s->d_desc + n * 8), d_out, n, s->st);
        if (rc)
            return rc;
    }
    if (hipMemcpyAsync(s->h_desc + n * 12, d_out, n * 4, hipMemcpyDeviceToHost, s->st) != hipSuccess ||
        hipStreamSynchronize(s->st) != hipSuccess)
        return ZDB_CRC32_ELAUNCH;
    std::memcpy(out, s->h_desc + n * 12, n * 4);
    return ZDB_CRC32_OK;
}

void zdb_crc32_stream_close(zdb_crc32_stream_t *s) { stream_free(s); }

int zdb_synth_fill_device(uint8_t *d_buf, size_t len, uint64_t seed, void *stream) {
    if (!len)
        return ZDB_CRC32_OK;
    if (!d_buf || (reinterpret_cast<uintptr_t>(d_buf) & 7))
        return ZDB_CRC32_EINVAL;
    g_hip_touched = true;
    hipLaunchKernelGGL(synth_kernel, dim3(8192), dim3(256), 0, static_cast<hipStream_t>(stream), d_buf,
                       (uint64_t)len, seed);
    return hipGetLastError() == hipSuccess ? ZDB_CRC32_OK : ZDB_CRC32_ELAUNCH;
}

} // extern "C"
