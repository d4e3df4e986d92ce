// Native (C++17) data-pipeline index builders for scaling_amd.
//
// * blended_sample: replaces the reference's Rust `blended_dataset_loop.sample(counts, stem)`
//   (src/scaling/core/data/blended_dataset.py:316-329).  Greedy interleave: the next sample comes
//   from the dataset whose sampled/target ratio is smallest (ties -> lowest dataset index), until
//   EVERY dataset reached its target (output length = sum(counts)).  O(N log D) with a binary heap
//   and exact rational comparisons.  Writes {stem}.bin (int64 [N, 2] rows (dataset, index)),
//   {stem}.meta.json and {stem}.input.json.
// * text_index: the TextDataset item index (src/scaling/transformer/data/text_dataset.py:223-335):
//   packs shuffled documents into items of exactly seq_len+1 tokens as (doc, start, end) triples,
//   incl. the only_full_sequences / allow_incomplete_sequences_every_n policy.  The document order
//   (numpy RandomState shuffle) is produced by the caller so the result is bit-identical.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <cstdio>
#include <fstream>
#include <queue>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

struct Entry {
    int64_t sampled, target;
    int64_t ds;
};
// "a has lower priority than b" for std::priority_queue (max-heap) => we want min ratio first.
struct Worse {
    bool operator()(const Entry& a, const Entry& b) const {
        // ratio a = a.sampled / a.target ; compare a > b  (so smaller ratio pops first)
        const __int128 l = (__int128)a.sampled * b.target, r = (__int128)b.sampled * a.target;
        if (l != r) return l > r;
        return a.ds > b.ds;  // tie: lower dataset index first
    }
};

int64_t blended_sample(py::array_t<int64_t, py::array::c_style | py::array::forcecast> counts, const std::string& stem) {
    auto c = counts.unchecked<1>();
    const int64_t n = c.shape(0);
    if (n <= 0) throw std::invalid_argument("blended_sample: need at least one dataset");
    int64_t total = 0;
    std::priority_queue<Entry, std::vector<Entry>, Worse> pq;
    for (int64_t i = 0; i < n; ++i) {
        if (c(i) <= 0) throw std::invalid_argument("blended_sample: counts must be positive");
        total += c(i);
        pq.push({0, c(i), i});
    }
    std::vector<int64_t> out;
    out.reserve((size_t)total * 2);
    {
        py::gil_scoped_release nogil;
        while (!pq.empty()) {
            Entry e = pq.top();
            pq.pop();
            out.push_back(e.ds);
            out.push_back(e.sampled);
            e.sampled += 1;
            if (e.sampled < e.target) pq.push(e);
        }
    }
    {
        std::ofstream f(stem + ".bin", std::ios::binary);
        f.write(reinterpret_cast<const char*>(out.data()), (std::streamsize)(out.size() * sizeof(int64_t)));
        if (!f) throw std::runtime_error("blended_sample: cannot write " + stem + ".bin");
    }
    {
        std::ofstream f(stem + ".input.json");
        f << "{\"number_to_sample_by_dataset\": [";
        for (int64_t i = 0; i < n; ++i) f << (i ? ", " : "") << c(i);
        f << "]}";
    }
    {
        // meta last: readers treat it as the completion marker
        std::ofstream f(stem + ".meta.json.tmp");
        f << "{\"dtype\": \"int64\", \"shape\": [" << total << ", 2]}";
        f.close();
        std::rename((stem + ".meta.json.tmp").c_str(), (stem + ".meta.json").c_str());
    }
    return total;
}

// Returns (flat triples int64, per-item (start, length) int64 pairs) as numpy arrays.
py::tuple text_index(py::array_t<int64_t, py::array::c_style | py::array::forcecast> doc_sizes,
                     py::array_t<int64_t, py::array::c_style | py::array::forcecast> doc_order, int64_t seq_len,
                     bool only_full_sequences, int64_t allow_incomplete_every_n) {
    auto sz = doc_sizes.unchecked<1>();
    auto order = doc_order.unchecked<1>();
    std::vector<int64_t> data, index;
    {
        py::gil_scoped_release nogil;
        std::vector<int64_t> item;
        int64_t item_tokens = 0, full = 0, half = 0, pos_total = 0;
        bool in_half = false;
        for (int64_t oi = 0; oi < order.shape(0); ++oi) {
            const int64_t doc = order(oi);
            const int64_t count = sz(doc);
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
    py::array_t<int64_t> d((py::ssize_t)data.size()), ix((py::ssize_t)index.size());
    std::copy(data.begin(), data.end(), d.mutable_data());
    std::copy(index.begin(), index.end(), ix.mutable_data());
    return py::make_tuple(d, ix);
}

}  // namespace

PYBIND11_MODULE(_data, m) {
    m.doc() = "scaling_amd native data-pipeline index builders (C++17)";
    m.def("blended_sample", &blended_sample, py::arg("counts"), py::arg("stem"));
    m.def("text_index", &text_index, py::arg("doc_sizes"), py::arg("doc_order"), py::arg("seq_len"),
          py::arg("only_full_sequences") = false, py::arg("allow_incomplete_every_n") = 0);
}
