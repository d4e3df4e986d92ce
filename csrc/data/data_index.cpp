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

#include "data_index_core.h"

namespace py = pybind11;

namespace {

int64_t blended_sample(py::array_t<int64_t, py::array::c_style | py::array::forcecast> counts, const std::string& stem) {
    auto c = counts.unchecked<1>();
    const int64_t n = c.shape(0);
    std::vector<int64_t> out;
    {
        py::gil_scoped_release nogil;
        out = scaling_data::blended_order(counts.data(), n);
    }
    const int64_t total = (int64_t)out.size() / 2;
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
    std::vector<int64_t> data, index;
    {
        py::gil_scoped_release nogil;
        scaling_data::text_index(doc_sizes.data(), doc_sizes.shape(0), doc_order.data(), doc_order.shape(0), seq_len,
                                 only_full_sequences, allow_incomplete_every_n, data, index);
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
