// Pure C++17 cores of the data-pipeline index builders (no Python / pybind11), shared by the
// `_data` extension (data_index.cpp) and the host sanitizer harness (data_index_asan.cpp).
// See data_index.cpp for the behaviour each function reproduces.
#pragma once

#include <algorithm>
#include <cstdint>
#include <queue>
#include <stdexcept>
#include <string>
#include <vector>

namespace scaling_data {

struct Entry {
    int64_t sampled, target;
    int64_t ds;
};
// max-heap comparator: the entry with the smallest sampled/target ratio pops first
struct Worse {
    bool operator()(const Entry& a, const Entry& b) const {
        const __int128 l = (__int128)a.sampled * b.target, r = (__int128)b.sampled * a.target;
        if (l != r) return l > r;
        return a.ds > b.ds;  // tie: lower dataset index first
    }
};

// Greedy interleave -> flat (dataset, index) pairs, length 2 * sum(counts).
inline std::vector<int64_t> blended_order(const int64_t* counts, int64_t n) {
    if (n <= 0) throw std::invalid_argument("blended_sample: need at least one dataset");
    int64_t total = 0;
    std::priority_queue<Entry, std::vector<Entry>, Worse> pq;
    for (int64_t i = 0; i < n; ++i) {
        if (counts[i] <= 0) throw std::invalid_argument("blended_sample: counts must be positive");
        total += counts[i];
        pq.push({0, counts[i], i});
    }
    std::vector<int64_t> out;
    out.reserve((size_t)total * 2);
    while (!pq.empty()) {
        Entry e = pq.top();
        pq.pop();
        out.push_back(e.ds);
        out.push_back(e.sampled);
        e.sampled += 1;
        if (e.sampled < e.target) pq.push(e);
    }
    return out;
}

// TextDataset item index: (doc, start, end) triples in `data`, per-item (offset, length) in `index`.
inline void text_index(const int64_t* sz, int64_t n_docs, const int64_t* order, int64_t n_order, int64_t seq_len,
                       bool only_full_sequences, int64_t allow_incomplete_every_n, std::vector<int64_t>& data,
                       std::vector<int64_t>& index) {
    if (seq_len <= 0) throw std::invalid_argument("text_index: seq_len must be positive");
    std::vector<int64_t> item;
    int64_t item_tokens = 0, full = 0, half = 0, pos_total = 0;
    bool in_half = false;
    for (int64_t oi = 0; oi < n_order; ++oi) {
        const int64_t doc = order[oi];
        if (doc < 0 || doc >= n_docs) throw std::out_of_range("text_index: document id out of range");
        const int64_t count = sz[doc];
        int64_t pos = 0;
        while (pos < count - 1) {
            const int64_t end = std::min(count, pos + 1 + seq_len - item_tokens);
            if (only_full_sequences) {
                if (in_half) {
                } else if (end - pos < seq_len + 1) {
                    if (allow_incomplete_every_n != 0 &&
                        ((double)full / (double)allow_incomplete_every_n - (double)half) >= 1.0) {
                        in_half = true;
                    } else {
                        break;
                    }
                } else {
                    full += 1;
                }
            }
            item_tokens += end - pos;
            item.push_back(doc);
            item.push_back(pos);
            item.push_back(end);
            if (item_tokens == seq_len + 1) {
                index.push_back(pos_total);
                index.push_back((int64_t)item.size());
                pos_total += (int64_t)item.size();
                data.insert(data.end(), item.begin(), item.end());
                item.clear();
                item_tokens = 0;
                if (in_half) half += 1;
                in_half = false;
            }
            pos = end - 1;
        }
    }
}

}  // namespace scaling_data
