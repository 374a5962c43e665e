// kg_internal.h -- shared definitions of libketogpu (host + device).
//
// HBM layout of a snapshot (all arrays device-resident, built once, immutable afterwards):
//   adj_off[n_nodes+1] u64 / adj[] u32   set-adjacency: per node (ns,obj,rel) the subject-set
//                                        subjects that checkExpandSubject recurses into
//                                        (internal/check/engine.go:118-136: SubjectIDs and "..."
//                                        sets skipped), kept in shard_id order.
//   row_off[n_nodes+1] u64 / row_subj[]   full rows (every subject, tagged), shard_id order: expand
//                                        (internal/expand/engine.go:57-94) and tuple-to-subject-set.
//   crow_off / crow_subj                  check rows (rewrite materialisation, kg_augment.hip): the
//                                        direct tuples checkDirect sees per node -- a materialised
//                                        union node holds the rows of every relation it unites;
//                                        nullptr: the full rows.  dset, signatures and holders use them.
//   dset                                  bucketed hash set of (node << 32 | tagged subject):
//                                        checkDirect's exact-tuple query (engine.go:159-163).
//   nmap                                  (ns,rel,obj) -> node id + its set row (begin, length), one
//                                        32-B slot per key, for request mapping on device.
//   nflags[n_nodes] u8                    bit0 IMPURE: a rewrite / undeclared relation is reachable
//                                        through set-adjacency (needs the rewrite interpreter).
//   radj_off[n_nodes+1] u64 / radj[] u32  reverse set-adjacency (parents), for the backward tier.
//   hold[] u32 + subject hash             holders: the nodes whose row contains a given subject,
//   hbits[] u32                           holder bitmap over subject ids (k_resolve's no-holder test)
//                                        grouped by subject (the backward tier's level 0).
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#define __host__
#define __device__
#define __forceinline__ inline
#endif

namespace kg {

constexpr uint32_t SET_BIT = 0x80000000u;
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint64_t EMPTY64 = ~0ull;
// u64 keys per dset bucket: 2 = one 16-B load per probe.  The unit of cost of these kernels is the
// random lane-request (tools/randprobe: ~41 G/s from HBM-sized tables, whatever their width up to
// 16 B), so a probe is one request at load <= 0.25 rather than four 16-B loads of a 64-B bucket.
constexpr int DSET_BUCKET = 2;

enum : uint8_t { NF_IMPURE = 1, NF_REWRITE = 2, NF_ERR = 4 };

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

__host__ __device__ __forceinline__ uint64_t nmap_key(uint32_t ns, uint32_t rel, uint32_t obj) {
  return ((uint64_t)((ns << 16) | (rel & 0xFFFFu)) << 32) | obj;
}
__host__ __device__ __forceinline__ uint64_t dset_key(uint32_t node, uint32_t subj) {
  return ((uint64_t)node << 32) | subj;
}
// Home slot of a key in an open-addressing table of n slots (dset buckets, node map): multiply-shift
// range reduction over any n, so a table is sized for its load exactly instead of rounding up to a
// power of two (up to 2x the HBM).  Linear probing wraps with hash_next.
__host__ __device__ __forceinline__ uint64_t hash_home(uint64_t key, uint64_t n) {
  return (uint64_t)(((unsigned __int128)mix64(key) * n) >> 64);
}
__host__ __device__ __forceinline__ uint64_t hash_next(uint64_t i, uint64_t n) { return i + 1 == n ? 0 : i + 1; }
// dset home bucket of a (node << 32 | subject) key: multiply-shift (Fibonacci) hashing -- the key times
// an odd 64-bit constant, whose high bits mix every key bit, scaled to the bucket count by a 64 x 32 high
// product (n < 2^32: the table is capped below a fifth of HBM).  5 integer multiplies where mix64 plus a
// 128-bit product took 10: the stream tier spends most of its time issuing VALU (profiles/r4g_*), and
// this hash ran for every lane of every step.
__host__ __device__ __forceinline__ uint64_t dset_home(uint64_t key, uint64_t n) {
  const uint64_t x = key * 0x9E3779B97F4A7C15ull;
  return ((x >> 32) * n + (((x & 0xFFFFFFFFull) * n) >> 32)) >> 32;
}

// Owner of position i in a CSR with offsets off[0..n]: the last node whose row starts at or before i
// (empty rows share a start; the owner is the one whose range holds i).  Lets the build kernels run
// one thread per row entry: a thread per node waits for the longest (hub) row.
__host__ __device__ __forceinline__ uint32_t csr_owner_from(const uint64_t* off, uint32_t lo, uint32_t n, uint64_t i) {
  uint32_t hi = n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (off[mid] <= i) lo = mid;
    else hi = mid;
  }
  return lo;
}
__host__ __device__ __forceinline__ uint32_t csr_owner(const uint64_t* off, uint32_t n, uint64_t i) {
  return csr_owner_from(off, 0, n, i);
}
// Advances owner v (of some position < i) to the owner of position i: one step covers the common
// case (the next row), a search the rest (long runs of empty rows: C3 has blocks of 10^8 nodes
// without set-adjacency, which a step-by-step walk crossed in one thread for seconds).
__host__ __device__ __forceinline__ uint32_t csr_advance(const uint64_t* off, uint32_t n, uint32_t v, uint64_t i) {
  if (off[v + 1] > i) return v;
  if (off[v + 2] > i) return v + 1;
  return csr_owner_from(off, v + 1, n, i);
}

// Shard of a node in the hash-sharded mode: all relations of one object live on
// one rank, owner = hash(ns, obj) mod nranks.
__host__ __device__ __forceinline__ uint32_t shard_owner(uint32_t ns, uint32_t obj, uint32_t nranks) {
  return nranks <= 1 ? 0u : (uint32_t)((mix64(((uint64_t)ns << 32) | obj) >> 20) % nranks);
}

// Rewrite-program node (kg_rw_node layout).
struct RwNode {
  int32_t kind, rel, crel, first, count;
};
enum { RW_OR = 0, RW_AND = 1, RW_COMPUTED = 2, RW_TTU = 3, RW_NOT = 4 };

// Bloom signature of a node's direct subjects (its full row): 44 bits, 2 per subject.  A
// checkDirect probe whose subject bits are not all present is a certain miss and is skipped.  The
// bits sit in two words as they are stored: x = signature bits 0-11 in bits 20-31 (bits 0-19 hold
// the carrier's own low field: AdjX's row length, NSlot's flags), y = signature bits 12-43.
// (Round 3 had 32 bits: a row of 20 subjects passed 52 % of absent subjects, now 36 %.)
constexpr uint32_t SIG_LO = 0xFFF00000u;
__host__ __device__ __forceinline__ uint2 subj_sig(uint32_t subj) {
  uint32_t h = subj * 0x9E3779B1u;
  h ^= h >> 15;
  h *= 0x85EBCA77u;
  h ^= h >> 13;
  const uint32_t p0 = ((h & 0xFFFFu) * 44u) >> 16, p1 = ((h >> 16) * 44u) >> 16;  // two positions in [0, 44)
  uint2 m = make_uint2(0u, 0u);
  if (p0 < 12) m.x |= 1u << (20 + p0);
  else m.y |= 1u << (p0 - 12);
  if (p1 < 12) m.x |= 1u << (20 + p1);
  else m.y |= 1u << (p1 - 12);
  return m;
}
// sig_lo: a word whose bits 20-31 are signature bits 0-11 (bits 0-19 are ignored), sig_hi: bits 12-43
__host__ __device__ __forceinline__ bool sig_maybe(uint32_t sig_lo, uint32_t sig_hi, uint2 m) {
  return ((sig_lo & m.x) == m.x) & ((sig_hi & m.y) == m.y);
}

// One set-adjacency edge with the child's own set row inlined (begin / length) and the child's
// signature: a BFS level needs one dependent HBM round trip instead of two (no adj_off lookup per
// discovered node).  lsig: the row length in bits 0-19 (ADJX_LEN_SAT = 2^20 - 1 or longer: read
// adj_off, adjx_len) and signature bits 0-11 in bits 20-31; sig: signature bits 12-43.  20 bits keep
// hub rows exact (the heavy-tail point's 10^5-edge rows would otherwise cost every edge into a hub
// a dependent adj_off read in the grid tiers).
constexpr uint32_t ADJX_LEN_SAT = 0xFFFFFu;
struct AdjX {
  uint32_t node, begin, lsig, sig;
};
__host__ __device__ __forceinline__ uint32_t adjx_len16(const AdjX& x) { return x.lsig & ADJX_LEN_SAT; }

// Node-map slot: key (ns,rel,obj), node id and the node's set-adjacency row, one 32-B slot so a
// request mapping is one random line.  key == EMPTY64: free.
// A check row of at most NSLOT_INL subjects rides in the slot itself (round 6): the first in pad1's high
// word, the second in `sig` (such a row needs no Bloom signature) -- the root's checkDirect
// (engine.go:148-177) then reads no dset line.  Doc rows are that short for ~3/4 of the C2 roots.
// (A 64-B slot with up to 8 subjects cut k_resolve's fabric requests 10 % but cost the headline ~8 %:
// twice the node map's footprint, profiles/r6m_*.)
constexpr uint32_t NSLOT_INL = 2;
struct NSlot {
  uint64_t key;
  uint32_t node, beg, len;
  // signature bits 12-43 of the node's row subjects (as AdjX.sig): k_resolve's root probe filter; for an
  // inline row of two subjects, the second subject
  uint32_t sig;
  // bits 0-7: the node's flags (nflags; 0 without a namespace program); bits 8-9: 1 + the number of
  // inline check-row subjects (0: not inlined -- probe dset); bits 20-31: signature bits 0-11 (rows not
  // inlined); bits 32-63: the first inline subject
  uint64_t pad1;
};
static_assert(sizeof(NSlot) == 32, "one 32-B node-map slot");
__host__ __device__ __forceinline__ uint32_t nslot_inline(uint64_t pad1) { return (uint32_t)(pad1 >> 8) & 3u; }
// checkDirect against an inlined row (icnt = nslot_inline(pad1) >= 1): exact
__host__ __device__ __forceinline__ bool nslot_inline_has(uint32_t icnt, uint64_t pad1, uint32_t sig, uint32_t subj) {
  return (icnt >= 2 && (uint32_t)(pad1 >> 32) == subj) | (icnt == 3 && sig == subj);
}
// Holder-hash slot: tagged subject -> hold[first, first + count).  key == NONE: free.
struct HSlot {
  uint32_t key, first, count, pad;
};

// Everything a kernel needs, passed by value.
struct DevSnap {
  uint32_t n_nodes;
  uint32_t wildcard_rel;
  const uint64_t* adj_off;
  const uint32_t* adj;
  const AdjX* adjx;  // one record per set edge: parallel to adj, or laid out hot-first (adjx_off)
  const uint64_t* row_off;
  const uint32_t* row_subj;
  const uint64_t* crow_off;  // check rows (nullptr: row_off / row_subj)
  const uint32_t* crow_subj;
  const uint64_t* dset;
  uint64_t dset_nb;  // buckets (DSET_BUCKET keys each); probes wrap at dset_nb
  const NSlot* nmap;
  uint64_t nmap_n;  // slots
  const uint8_t* nflags;  // nullptr: every node pure
  const uint32_t* nd_ns;
  const uint32_t* nd_obj;
  const uint32_t* nd_rel;
  // program: relation flags [n_ns * n_rel] (bit0 has rewrite, bit1 undeclared->error), roots
  uint32_t n_ns, n_rel;
  const uint8_t* ns_has_rel;  // [n_ns]: configured with relations (unknown relation ids -> error)
  const uint8_t* relflags;
  const int32_t* relroot;
  const RwNode* rw;
  const int32_t* rwchild;
  uint32_t n_rw;
  const uint8_t* virt;  // [n_ns * n_rel]: 1 = a materialised union relation (kg_augment.hip), or nullptr
  // reverse indexes (backward tier, kg_check.hip k_back); radj == nullptr: not built
  const uint64_t* radj_off;  // [n_nodes+1] parents of a node through set-adjacency
  const uint32_t* radj;
  const uint32_t* hold;      // holder nodes (rows containing a subject), grouped by subject
  const HSlot* hslots;       // subject hash: tagged subject -> (first index into hold, count)
  uint64_t hmask;            // n_slots - 1
  const uint32_t* hbits;     // holder bitmap over subject ids: bit s set <=> some row holds subject id s
  uint32_t hbits_n;          // bits in hbits (max held subject id + 1); nullptr / 0: not built
  // hash-sharded mode: this snapshot holds the rows of the nodes with shard_owner == shard_rank
  uint32_t shard_rank, shard_n;
  const uint8_t* nowner;  // [n_nodes] owner rank of every node (shard_n > 1)
  // shard_n > 1, set when a transport is bound (kg_shard_comm.hip comm_setup): an adjx record whose
  // child another rank owns has begin = ADJX_REMOTE | owner and the OWNER's row length and signature
  // in lsig / sig (all-reduced at bind time), so the sender decides like for a local child -- no
  // nowner read per edge, and a remote child that can neither hit nor expand is never sent
  uint32_t remote_meta;
  // adjx laid out hot-first (kg_snapshot.hip build_hash_tables): the adjx begin of every node's set
  // row -- what nmap slots and adjx records carry; adj_off still gives lengths and the adj rows.
  // nullptr: adjx is parallel to adj (begin = adj_off)
  const uint32_t* adjx_off;
};
constexpr uint32_t ADJX_REMOTE = 0x80000000u;

// The child's exact set-row length (one adj_off read for rows of ADJX_LEN_SAT edges or more).
__device__ __forceinline__ uint32_t adjx_len(const DevSnap& s, const AdjX& x) {
  const uint32_t l = adjx_len16(x);
  return l < ADJX_LEN_SAT ? l : (uint32_t)(s.adj_off[x.node + 1] - s.adj_off[x.node]);
}

// astRelationFor (internal/check/engine.go:209-229) as flags: bit0 = has rewrite, bit1 = the
// namespace is configured with relations and this one is not declared ("relation %q not found").
// Unknown namespaces and namespaces without relations accept every relation without rewrite.
__host__ __device__ __forceinline__ uint8_t relflag(const DevSnap& s, uint32_t ns, uint32_t rel) {
  if (!s.relflags || ns >= s.n_ns) return 0;
  if (rel >= s.n_rel) return s.ns_has_rel[ns] ? 2 : 0;
  return s.relflags[(size_t)ns * s.n_rel + rel];
}

// Resolved query as stored in HBM by the mapping kernel.
struct RQuery {
  uint32_t node;   // root node id or NONE
  uint32_t subj;   // tagged subject or NONE
  int32_t depth;   // clamped rest depth
  uint32_t route;  // ROUTE_*
  uint32_t beg, len;  // root's set-adjacency row
};
enum : uint32_t { ROUTE_DONE = 0, ROUTE_LIGHT = 1, ROUTE_GENERAL = 2 };

// A light-routed query as k_resolve appends it to the stream tier's work list (k_stream4): the
// resolved query travels with its list entry, so k_resolve writes it once, contiguously (no
// scattered 24-B rq[i] store), and a stream-tier dequeue is one coalesced read (no list -> rq hop).
struct LQuery {
  uint32_t qi;     // query index in the batch
  uint32_t node;   // root node
  uint32_t subj;   // tagged subject
  int32_t depth;   // clamped rest depth
  uint32_t beg, len;  // root's set-adjacency row
};

}  // namespace kg
