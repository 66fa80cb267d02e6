// lp_io.h — LP file formats of the ./solver CLI.
//
// Text: the reference's format (input/sample.txt; reader at
// src/v4_cub_reduction.cu:94-104,401-419): "m n", A (m x n row-major), b (m),
// c (n), whitespace separated; anything after c is ignored.  Parsed in
// parallel: the file is read once, split at whitespace into per-thread chunks,
// tokens are counted, then parsed straight into their column-major slots.
//
// Binary (".spxlp"): 8-byte magic "SPXLP001", int64 m,
// int64 n, then A column-major (m*n doubles), b (m), c (n), little-endian.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace lpio {

struct LP {
    int64_t m = 0, n = 0;
    std::vector<double> A;  // column-major, A[i + j*m]
    std::vector<double> b, c;
};

constexpr char kMagic[8] = {'S', 'P', 'X', 'L', 'P', '0', '0', '1'};

// 0 on success; otherwise err holds the reference's message where it has one
// ("Either failed to read m and n, or m > n.", "Failed to read (i,j) for A").
int read_any(const std::string& path, LP& lp, std::string& err, int threads = 0);
int read_text(const std::string& path, LP& lp, std::string& err, int threads = 0);
int read_binary(const std::string& path, LP& lp, std::string& err);
int write_binary(const std::string& path, const LP& lp, std::string& err);
// trailer: text appended after c (the reference's reader ignores it, v4:94-104)
int write_text(const std::string& path, const LP& lp, std::string& err, const std::string& trailer = "");
bool is_binary(const std::string& path);

// Host copy of the seeded LP of SURVEY.md §8(d), bit-identical to the device
// generator (k_generate): lets `--gen m n seed --write-bin f` export it.
void generate(int64_t m, int64_t n, uint64_t seed, LP& lp);

}  // namespace lpio
