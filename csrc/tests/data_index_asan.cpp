// Host sanitizer harness for the data-pipeline index builders (csrc/data/data_index_core.h).
// Built by tests/test_host_sanitizers.py with -fsanitize=address,undefined and run standalone (no
// Python in the process, so ASan/UBSan see every heap access of the C++ cores).  Exits non-zero on a
// wrong result; the sanitizers abort on any memory or UB error.
#include <cstdio>
#include <random>
#include <vector>

#include "../data/data_index_core.h"

static int fail(const char* what) {
    std::fprintf(stderr, "FAIL: %s\n", what);
    return 1;
}

int main() {
    std::mt19937_64 rng(1234);
    // blended order: every dataset reaches exactly its target, indices are 0..count-1 in order
    for (int trial = 0; trial < 50; ++trial) {
        const int n = 1 + (int)(rng() % 7);
        std::vector<int64_t> counts(n);
        for (auto& c : counts) c = 1 + (int64_t)(rng() % 500);
        const auto out = scaling_data::blended_order(counts.data(), n);
        std::vector<int64_t> seen(n, 0);
        for (size_t i = 0; i < out.size(); i += 2) {
            const int64_t ds = out[i];
            if (ds < 0 || ds >= n) return fail("dataset id range");
            if (out[i + 1] != seen[ds]) return fail("per-dataset index order");
            seen[ds] += 1;
        }
        for (int i = 0; i < n; ++i)
            if (seen[i] != counts[i]) return fail("dataset target count");
    }
    // text index: every item spans exactly seq_len+1 tokens with one-token overlap between pieces
    for (int trial = 0; trial < 50; ++trial) {
        const int64_t n_docs = 1 + (int64_t)(rng() % 200), seq_len = 1 + (int64_t)(rng() % 64);
        std::vector<int64_t> sizes(n_docs), order(n_docs);
        for (int64_t i = 0; i < n_docs; ++i) {
            sizes[i] = (int64_t)(rng() % 300);
            order[i] = i;
        }
        std::shuffle(order.begin(), order.end(), rng);
        for (int mode = 0; mode < 3; ++mode) {
            std::vector<int64_t> data, index;
            scaling_data::text_index(sizes.data(), n_docs, order.data(), n_docs, seq_len, mode > 0, mode == 2 ? 3 : 0,
                                     data, index);
            for (size_t it = 0; it < index.size(); it += 2) {
                const int64_t off = index[it], len = index[it + 1];
                if (off < 0 || len <= 0 || len % 3 || off + len > (int64_t)data.size()) return fail("item bounds");
                int64_t tokens = 0;
                for (int64_t j = off; j < off + len; j += 3) {
                    const int64_t doc = data[j], s = data[j + 1], e = data[j + 2];
                    if (doc < 0 || doc >= n_docs || s < 0 || e > sizes[doc] || e <= s) return fail("piece bounds");
                    tokens += e - s;
                }
                if (tokens != seq_len + 1) return fail("item length");
            }
        }
        // invalid document ids are rejected, never read out of bounds
        std::vector<int64_t> bad = {0, n_docs};
        std::vector<int64_t> d, ix;
        bool threw = false;
        try {
            scaling_data::text_index(sizes.data(), n_docs, bad.data(), 2, seq_len, false, 0, d, ix);
        } catch (const std::out_of_range&) {
            threw = true;
        }
        if (!threw) return fail("out-of-range document id accepted");
    }
    std::printf("data_index sanitizer harness ok\n");
    return 0;
}
