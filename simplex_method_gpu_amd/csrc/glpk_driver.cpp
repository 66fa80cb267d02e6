// glpk_driver.cpp — `solver_glpk`: the counterpart of the reference's GLPK CPU
// driver (solver_glpk.cpp:1-43), SURVEY.md §8c/§8f row 2.
//
// libglpk is not installed in this image (nor on the GPU box), and no GLPK
// header is vendored, so the library is bound at run time with dlopen/dlsym
// against the few C entry points the reference calls.  Without libglpk the
// driver prints "GLPK unavailable" on stderr and exits 3 — it never
// substitutes another solver.  With it:
//   solver_glpk file.mps            fixed MPS (GLP_MPS_DECK, solver_glpk.cpp:15),
//                                   default minimisation, glp_simplex(lp, NULL)
//   solver_glpk --free file.mps     free MPS (GLP_MPS_FILE, glpk_interface.cpp:22)
//   solver_glpk --text file.txt     the solver's text LP (v4:94-104) as
//                                   max c x, A x = b, x >= 0 (GLP_MAX) — the
//                                   dense random LPs of the benchmark
// Output as the reference: "x[i] = v" per column and "Optimal objective: z",
// or "Problem status: <code>"; plus "Iterations: k" and "Simplex seconds: t"
// (steady clock around glp_simplex only).
#include <dlfcn.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "lp_io.h"

namespace {

struct Glpk {
    void* h = nullptr;
    void* (*create_prob)() = nullptr;
    void (*set_prob_name)(void*, const char*) = nullptr;
    int (*read_mps)(void*, int, const void*, const char*) = nullptr;
    int (*simplex)(void*, const void*) = nullptr;
    int (*get_status)(void*) = nullptr;
    int (*get_num_cols)(void*) = nullptr;
    double (*get_obj_val)(void*) = nullptr;
    double (*get_col_prim)(void*, int) = nullptr;
    void (*delete_prob)(void*) = nullptr;
    int (*term_out)(int) = nullptr;
    void (*set_obj_dir)(void*, int) = nullptr;
    int (*add_rows)(void*, int) = nullptr;
    int (*add_cols)(void*, int) = nullptr;
    void (*set_row_bnds)(void*, int, int, double, double) = nullptr;
    void (*set_col_bnds)(void*, int, int, double, double) = nullptr;
    void (*set_obj_coef)(void*, int, double) = nullptr;
    void (*load_matrix)(void*, int, const int*, const int*, const double*) = nullptr;
    int (*get_it_cnt)(void*) = nullptr;  // optional (newer GLPK)

    template <typename F>
    bool sym(F& f, const char* name, bool required = true) {
        f = reinterpret_cast<F>(dlsym(h, name));
        return f || !required;
    }
    bool load() {
        for (const char* so : {"libglpk.so", "libglpk.so.40", "libglpk.so.36", "libglpk.so.35"}) {
            h = dlopen(so, RTLD_NOW | RTLD_LOCAL);
            if (h) break;
        }
        if (!h) return false;
        return sym(create_prob, "glp_create_prob") && sym(set_prob_name, "glp_set_prob_name") &&
               sym(read_mps, "glp_read_mps") && sym(simplex, "glp_simplex") && sym(get_status, "glp_get_status") &&
               sym(get_num_cols, "glp_get_num_cols") && sym(get_obj_val, "glp_get_obj_val") &&
               sym(get_col_prim, "glp_get_col_prim") && sym(delete_prob, "glp_delete_prob") &&
               sym(term_out, "glp_term_out") && sym(set_obj_dir, "glp_set_obj_dir") &&
               sym(add_rows, "glp_add_rows") && sym(add_cols, "glp_add_cols") &&
               sym(set_row_bnds, "glp_set_row_bnds") && sym(set_col_bnds, "glp_set_col_bnds") &&
               sym(set_obj_coef, "glp_set_obj_coef") && sym(load_matrix, "glp_load_matrix") &&
               sym(get_it_cnt, "glp_get_it_cnt", false);
    }
};

// glpk.h constants (stable across GLPK 4.x / 5.x)
constexpr int GLP_MAX = 2, GLP_FX = 5, GLP_LO = 2, GLP_OPT = 5, GLP_OFF = 0;
constexpr int GLP_MPS_DECK = 1, GLP_MPS_FILE = 2;

}  // namespace

int main(int argc, char* argv[]) {
    bool text = false, free_mps = false;
    const char* path = nullptr;
    for (int a = 1; a < argc; ++a) {
        const std::string s = argv[a];
        if (s == "--text") text = true;
        else if (s == "--free") free_mps = true;
        else if (!path) path = argv[a];
        else path = nullptr;
    }
    if (!path) {
        std::cerr << "Usage: " << argv[0] << " [--text | --free] file\n";
        return 1;
    }
    Glpk g;
    if (!g.load()) {
        std::cerr << "GLPK unavailable: libglpk.so could not be loaded (" << (dlerror() ? "dlopen failed" : "missing symbols")
                  << "); no substitute solver is used\n";
        return 3;
    }
    g.term_out(GLP_OFF);
    void* lp = g.create_prob();
    g.set_prob_name(lp, path);
    if (text) {
        lpio::LP t;
        std::string err;
        if (lpio::read_any(path, t, err) != 0) {
            std::cerr << err << "\n";
            g.delete_prob(lp);
            return 2;
        }
        g.set_obj_dir(lp, GLP_MAX);
        g.add_rows(lp, (int)t.m);
        g.add_cols(lp, (int)t.n);
        for (int64_t i = 0; i < t.m; ++i) g.set_row_bnds(lp, (int)i + 1, GLP_FX, t.b[(size_t)i], t.b[(size_t)i]);
        std::vector<int> ia(1), ja(1);
        std::vector<double> ar(1);
        for (int64_t j = 0; j < t.n; ++j) {
            g.set_col_bnds(lp, (int)j + 1, GLP_LO, 0.0, 0.0);
            g.set_obj_coef(lp, (int)j + 1, t.c[(size_t)j]);
            for (int64_t i = 0; i < t.m; ++i) {
                const double v = t.A[(size_t)(i + j * t.m)];
                if (v != 0.0) {
                    ia.push_back((int)i + 1);
                    ja.push_back((int)j + 1);
                    ar.push_back(v);
                }
            }
        }
        g.load_matrix(lp, (int)ia.size() - 1, ia.data(), ja.data(), ar.data());
    } else {
        const int err = g.read_mps(lp, free_mps ? GLP_MPS_FILE : GLP_MPS_DECK, nullptr, path);
        if (err != 0) {
            std::cerr << "Error reading MPS file: " << err << "\n";
            g.delete_prob(lp);
            return 2;
        }
    }
    const auto t0 = std::chrono::steady_clock::now();
    g.simplex(lp, nullptr);
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const int status = g.get_status(lp);
    if (status == GLP_OPT) {
        const int n = g.get_num_cols(lp);
        for (int i = 1; i <= n; ++i) std::cout << "x[" << i << "] = " << g.get_col_prim(lp, i) << "\n";
        std::cout << "Optimal objective: " << g.get_obj_val(lp) << "\n";
    } else {
        std::cout << "Problem status: " << status << "\n";
    }
    if (g.get_it_cnt) std::cout << "Iterations: " << g.get_it_cnt(lp) << "\n";
    std::cout << "Simplex seconds: " << sec << "\n";
    g.delete_prob(lp);
    return 0;
}
