// lp_io.cpp — text and binary LP readers/writers of the ./solver CLI (see lp_io.h).
#include "lp_io.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace lpio {
namespace {

inline bool is_space(char ch) { return ch == ' ' || ch == '\n' || ch == '\t' || ch == '\r' || ch == '\f' || ch == '\v'; }

struct Mapped {
    const char* data = nullptr;
    size_t size = 0;
    int fd = -1;
    ~Mapped() {
        if (data && size) munmap(const_cast<char*>(data), size);
        if (fd >= 0) close(fd);
    }
    bool open_file(const std::string& path) {
        fd = ::open(path.c_str(), O_RDONLY);
        if (fd < 0) return false;
        struct stat sb;
        if (fstat(fd, &sb) != 0) return false;
        size = (size_t)sb.st_size;
        if (size == 0) return true;
        void* p = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (p == MAP_FAILED) {
            size = 0;
            return false;
        }
        madvise(p, size, MADV_SEQUENTIAL);
        data = static_cast<const char*>(p);
        return true;
    }
};

// One whitespace-delimited token starting at p (< end); returns its end.
inline const char* token_end(const char* p, const char* end) {
    while (p < end && !is_space(*p)) ++p;
    return p;
}

// Parse [p, q) as a double; false unless the whole token is a number.
inline bool parse_double(const char* p, const char* q, double* out) {
    char buf[64];
    const size_t len = (size_t)(q - p);
    if (len == 0 || len >= sizeof(buf)) return false;  // numbers are short; prose may be long
    std::memcpy(buf, p, len);
    buf[len] = '\0';
    char* e = nullptr;
    errno = 0;
    const double v = std::strtod(buf, &e);
    if (e != buf + len) return false;
    *out = v;
    return true;
}

std::string fail_message(int64_t t, int64_t m, int64_t n) {
    // index t among the numbers after "m n": A row-major, then b, then c
    char buf[128];
    if (t < m * n)
        std::snprintf(buf, sizeof(buf), "Failed to read (%" PRId64 ",%" PRId64 ") for A", t / n, t % n);
    else if (t < m * n + m)
        std::snprintf(buf, sizeof(buf), "Failed to read (%" PRId64 ",0) for b", t - m * n);
    else
        std::snprintf(buf, sizeof(buf), "Failed to read (0,%" PRId64 ") for c", t - m * n - m);
    return buf;
}

}  // namespace

bool is_binary(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    char head[8];
    const bool ok = std::fread(head, 1, 8, f) == 8 && std::memcmp(head, kMagic, 8) == 0;
    std::fclose(f);
    return ok;
}

int read_text(const std::string& path, LP& lp, std::string& err, int threads) {
    Mapped mp;
    if (!mp.open_file(path)) {
        err = "Could not open " + path + ".";
        return 1;
    }
    const char* p = mp.data;
    const char* end = mp.data + mp.size;
    // header "m n" (v4:401-405)
    int64_t hdr[2];
    for (int h = 0; h < 2; ++h) {
        while (p < end && is_space(*p)) ++p;
        const char* q = token_end(p, end);
        char* e = nullptr;
        std::string tok(p, q);
        const long long v = std::strtoll(tok.c_str(), &e, 10);
        if (p == q || *e != '\0') {
            err = "Either failed to read m and n, or m > n.";
            return 1;
        }
        hdr[h] = v;
        p = q;
    }
    const int64_t m = hdr[0], n = hdr[1];
    if (m > n || m < 0) {
        err = "Either failed to read m and n, or m > n.";
        return 1;
    }
    const int64_t need = m * n + m + n;
    lp.m = m;
    lp.n = n;
    lp.A.assign((size_t)(m * n), 0.0);
    lp.b.assign((size_t)m, 0.0);
    lp.c.assign((size_t)n, 0.0);

    int T = threads > 0 ? threads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    const size_t span = (size_t)(end - p);
    if (span < (size_t)T * (1u << 20)) T = std::max<int>(1, (int)(span >> 20));  // >= 1 MiB per thread
    // chunk boundaries at token starts
    std::vector<const char*> cut((size_t)T + 1);
    cut[0] = p;
    cut[(size_t)T] = end;
    for (int t = 1; t < T; ++t) {
        const char* c = p + span * (size_t)t / (size_t)T;
        if (c < cut[(size_t)t - 1]) c = cut[(size_t)t - 1];
        while (c < end && !is_space(*c)) ++c;  // to the end of the token we landed in
        cut[(size_t)t] = c;
    }
    // pass 1: tokens per chunk
    std::vector<int64_t> count((size_t)T, 0);
    auto counter = [&](int t) {
        int64_t k = 0;
        const char* a = cut[(size_t)t];
        const char* b = cut[(size_t)t + 1];
        while (a < b) {
            while (a < b && is_space(*a)) ++a;
            if (a >= b) break;
            a = token_end(a, b);
            ++k;
        }
        count[(size_t)t] = k;
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < T; ++t) pool.emplace_back(counter, t);
    for (auto& th : pool) th.join();
    pool.clear();
    std::vector<int64_t> first((size_t)T + 1, 0);
    for (int t = 0; t < T; ++t) first[(size_t)t + 1] = first[(size_t)t] + count[(size_t)t];
    // pass 2: parse into the column-major slots (R2C, v4:59-60)
    std::atomic<int64_t> bad{INT64_MAX};
    auto parser = [&](int t) {
        int64_t k = first[(size_t)t];
        if (k >= need) return;
        const char* a = cut[(size_t)t];
        const char* b = cut[(size_t)t + 1];
        while (a < b && k < need) {
            while (a < b && is_space(*a)) ++a;
            if (a >= b) break;
            const char* q = token_end(a, b);
            double v;
            if (!parse_double(a, q, &v)) {
                int64_t cur = bad.load();
                while (k < cur && !bad.compare_exchange_weak(cur, k)) {
                }
                return;
            }
            if (k < m * n)
                lp.A[(size_t)((k / n) + (k % n) * m)] = v;
            else if (k < m * n + m)
                lp.b[(size_t)(k - m * n)] = v;
            else
                lp.c[(size_t)(k - m * n - m)] = v;
            ++k;
            a = q;
        }
    };
    for (int t = 0; t < T; ++t) pool.emplace_back(parser, t);
    for (auto& th : pool) th.join();
    const int64_t total = first[(size_t)T];
    const int64_t first_bad = std::min<int64_t>(bad.load(), total < need ? total : INT64_MAX);
    if (first_bad < need) {
        err = fail_message(first_bad, m, n);
        return 1;
    }
    return 0;
}

int read_binary(const std::string& path, LP& lp, std::string& err) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) {
        err = "Could not open " + path + ".";
        return 1;
    }
    char head[8];
    int64_t mn[2];
    if (std::fread(head, 1, 8, f) != 8 || std::memcmp(head, kMagic, 8) != 0 || std::fread(mn, 8, 2, f) != 2 ||
        mn[0] < 0 || mn[0] > mn[1]) {
        std::fclose(f);
        err = "Either failed to read m and n, or m > n.";
        return 1;
    }
    lp.m = mn[0];
    lp.n = mn[1];
    lp.A.resize((size_t)(lp.m * lp.n));
    lp.b.resize((size_t)lp.m);
    lp.c.resize((size_t)lp.n);
    const bool ok = std::fread(lp.A.data(), 8, lp.A.size(), f) == lp.A.size() &&
                    std::fread(lp.b.data(), 8, lp.b.size(), f) == lp.b.size() &&
                    std::fread(lp.c.data(), 8, lp.c.size(), f) == lp.c.size();
    std::fclose(f);
    if (!ok) {
        err = "truncated binary LP file " + path;
        return 1;
    }
    return 0;
}

int write_binary(const std::string& path, const LP& lp, std::string& err) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) {
        err = "Could not open " + path + " for writing.";
        return 1;
    }
    const int64_t mn[2] = {lp.m, lp.n};
    const bool ok = std::fwrite(kMagic, 1, 8, f) == 8 && std::fwrite(mn, 8, 2, f) == 2 &&
                    std::fwrite(lp.A.data(), 8, lp.A.size(), f) == lp.A.size() &&
                    std::fwrite(lp.b.data(), 8, lp.b.size(), f) == lp.b.size() &&
                    std::fwrite(lp.c.data(), 8, lp.c.size(), f) == lp.c.size();
    if (std::fclose(f) != 0 || !ok) {
        err = "write failed: " + path;
        return 1;
    }
    return 0;
}

int write_text(const std::string& path, const LP& lp, std::string& err, const std::string& trailer) {
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) {
        err = "Could not open " + path + " for writing.";
        return 1;
    }
    std::fprintf(f, "%" PRId64 " %" PRId64 "\n", lp.m, lp.n);
    for (int64_t i = 0; i < lp.m; ++i) {
        for (int64_t j = 0; j < lp.n; ++j)
            std::fprintf(f, j + 1 < lp.n ? "%.17g " : "%.17g\n", lp.A[(size_t)(i + j * lp.m)]);
    }
    for (int64_t i = 0; i < lp.m; ++i) std::fprintf(f, i + 1 < lp.m ? "%.17g " : "%.17g\n", lp.b[(size_t)i]);
    for (int64_t j = 0; j < lp.n; ++j) std::fprintf(f, j + 1 < lp.n ? "%.17g " : "%.17g\n", lp.c[(size_t)j]);
    if (!trailer.empty()) std::fputs(trailer.c_str(), f);
    if (std::fclose(f) != 0) {
        err = "write failed: " + path;
        return 1;
    }
    return 0;
}

namespace {
inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
inline double uniform01(uint64_t seed, uint64_t stream, uint64_t idx) {
    return (double)(splitmix64((seed * 0x9E3779B97F4A7C15ULL) ^ (stream << 56) ^ idx) >> 11) * 0x1.0p-53;
}
}  // namespace

void generate(int64_t m, int64_t n, uint64_t seed, LP& lp) {
    const int64_t ns = n - m;
    lp.m = m;
    lp.n = n;
    lp.A.assign((size_t)(m * n), 0.0);
    lp.b.resize((size_t)m);
    lp.c.assign((size_t)n, 0.0);
    for (int64_t j = 0; j < ns; ++j)
        for (int64_t i = 0; i < m; ++i) lp.A[(size_t)(i + j * m)] = uniform01(seed, 1, (uint64_t)(i + j * m));
    for (int64_t i = 0; i < m; ++i) lp.A[(size_t)(i + (ns + i) * m)] = 1.0;
    for (int64_t i = 0; i < m; ++i) lp.b[(size_t)i] = ((double)ns / 4.0) * (1.0 + uniform01(seed, 2, (uint64_t)i));
    for (int64_t j = 0; j < ns; ++j) lp.c[(size_t)j] = uniform01(seed, 3, (uint64_t)j);
}

int read_any(const std::string& path, LP& lp, std::string& err, int threads) {
    return is_binary(path) ? read_binary(path, lp, err) : read_text(path, lp, err, threads);
}

}  // namespace lpio
