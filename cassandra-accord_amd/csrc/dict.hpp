// dict.hpp — shared front end of the deps paths (keydeps.hip): input validation and the dense order-rank
// dictionary of every TxnId and executeAt of a batch (Timestamp.compareTo, primitives/Timestamp.java:208-217).
#pragma once

#include "prims.hpp"
#include <functional>

namespace acc {

struct Dictionary {
    uint32_t *rank = nullptr;         // [2n]: rank[t] = TxnId of t, rank[n + t] = executeAt of t
    uint32_t *txn_of_rank = nullptr;  // [2n]: txn index of each TxnId rank
    int rbits = 0;                    // bits of the largest rank
    bool batch_sorted = false;        // txns given in TxnId order
    bool fast = false;                // sorted-batch dictionary taken
    bool ties_pending = false;        // its executeAt-tie check (g[6]) is still to be read by the caller
    uint64_t hg[8] = {};              // prep words: ts word masks [0..2], key mask [3], errors [4], unsorted [5]
};

// Dense order ranks of n composite keys of nw (1..3) u64 words, most significant first, compared unsigned after
// (word & and_mask[k]) ^ xor_mask[k] (null masks: identity). rank[i] in [0, count); first[r] = smallest index of rank r
// (want_first). count is left on device (count_dev) for the caller's next sync. Buffers named "<tag>.*".
struct DenseRank {
    uint32_t *rank = nullptr;
    uint32_t *first = nullptr;
    const uint32_t *perm = nullptr;   // the stable sorted order of the n keys (nullptr: identity, every key equal)
    uint64_t *count_dev = nullptr;
    uint64_t count = 0;
};
DenseRank dense_rank(acc_ctx *ctx, const char *tag, size_t n, int nw, const uint64_t *const *words, const uint64_t *and_mask,
                     const uint64_t *xor_mask, bool want_first);

// key_off/key_code: the key-domain part (P pairs); owner[P] receives the txn of every pair; g[8] scratch words.
// the prep / dictionary flag words: g[0..7], then the prep pass's slotted partials (64 slots x 8 words), zeroed by one fill
constexpr size_t PREP_G_WORDS = 8 + 64 * 8;
void prep_dictionary(acc_ctx *ctx, uint32_t n, size_t P, const uint64_t *tm, const uint64_t *tl, const int32_t *tn,
                     const uint64_t *em, const uint64_t *el, const int32_t *en, const uint8_t *status,
                     const uint32_t *key_off, const uint64_t *key_code, uint32_t *owner, uint64_t *g, Dictionary &out,
                     bool defer_ties = false);
void redo_general_dictionary(acc_ctx *ctx, uint32_t n, const uint64_t *tm, const uint64_t *tl, const int32_t *tn,
                             const uint64_t *em, const uint64_t *el, const int32_t *en, uint64_t *g, Dictionary &d);

// The CommandsForKey snapshot of a key batch (keydeps.hip stages 1-3) for the scans other than mapReduceActive: pairs
// sorted by (key, TxnId rank) = one segment per key, entries in CommandsForKey.txns order. cfk = false when the batch has
// no pairs. Device pointers owned by the context, valid until its next compute call.
struct CfkSnapshot {
    bool cfk = false;
    uint32_t n = 0, nseg = 0;
    size_t P = 0;
    int rbits = 0;
    const uint32_t *rank = nullptr;         // [2n] dictionary ranks (TxnIds, then executeAts)
    const uint32_t *txn_of_rank = nullptr;  // TxnId rank -> batch index
    const uint32_t *seg_start = nullptr;    // [nseg] first entry of each segment
    const uint64_t *seg_key = nullptr;      // [nseg] key code of each segment, ascending
    const uint32_t *s_rank = nullptr, *s_exec = nullptr;   // [P] TxnId / executeAt rank per entry
    const uint8_t *s_info = nullptr;        // [P] status | kind << 3
    const uint32_t *perm = nullptr;         // [P] entry -> input pair index
    const uint64_t *tm = nullptr, *tl = nullptr, *em = nullptr, *el = nullptr;   // staged inputs
    const int32_t *tn = nullptr, *en = nullptr;
    const uint32_t *key_off = nullptr;
};
void cfk_snapshot(acc_ctx *ctx, const acc_batch_in *in, CfkSnapshot &out);

// The dictionary of a batch computed by one half of PartialDeps, handed to the other (acc_partial_deps_batch): valid
// when the KeyDeps half ran prep_dictionary (the batch has key pairs).
struct SharedDict {
    bool valid = false;
    Dictionary dict;
    const uint32_t *owner = nullptr;   // [P] txn of every key pair
    // called by keydeps_mixed once the dictionary is final (its kernels enqueued on the context stream): starts the
    // RangeDeps half concurrently with the rest of the KeyDeps half
    std::function<void(const SharedDict &)> ready;
};

}  // namespace acc
