// solver_main.cpp — `./solver <file>` CLI, the drop-in for the reference's
// bin/solverN.out (main() at src/v4_cub_reduction.cu:384-473).
//
// Same argv, same LP text format (m n, A row-major, b, c; trailing text
// ignored — reader at v4:94-104, 401-419), same stdout: "# Iteration k" per
// loop pass (v4:136-142), the result block (v4:426-445) and the timing table
// (v4:456-471).  Compute goes through libsimplex's C-ABI only.
//
// Extra flags (all optional, before the file):
//   --max-iter K   loop passes (default: unlimited; reference MAX_ITER=5, v4:19)
//   --eps E        optimality tolerance (default 1e-7; reference 1e-4 f32, v4:18)
//   --compat       reference constants: --max-iter 5 --eps 1e-4
//   --gen m n seed solve the seeded random LP of SURVEY.md §8(d) (no file)
//   --device D     HIP device ordinal
//   --no-iter-lines  suppress the "# Iteration k" lines
//   --json         also print one JSON result line
//   --threads T    text-parser threads (default: min(16, cores))
//   --write-bin F  write the loaded/generated LP as binary .spxlp (lp_io.h)
//   --write-text F write it in the reference's text format (%.17g, exact)
//   --no-solve     stop after reading/writing
//   --ratio R      leaving-row rule: reference | guarded | harris (simplex.h
//                  SPX_RATIO_*; default reference, guarded with --mps)
//   --piv-tol T, --feas-tol T   tolerances of the guarded / Harris rules
//   --refactor K   rebuild B^-1 from the basis every K pivots (spx_reinvert)
//   --window W     B^-1 representation (0 auto, -1 explicit, 8..64 eta window)
//   --pricing P    entering-column rule: dantzig (v4:288-302, default) | devex | steepest
//   --tableau      window tableau (SPX_FLAG_TABLEAU): T_w = B_w A
//                  kept in HBM, no per-pivot A / B^-1 stream
//   --mps          the input is an MPS file (mps_io.h): converted to the
//                  canonical form (slacks, senses, bounds, big-M artificials)
//                  and solved; output as the reference's GLPK driver
//                  (solver_glpk.cpp:27-38: "x[i] = v" per original column,
//                  "Optimal objective: z", else "Problem status: <GLPK code>");
//                  --write-text then writes the converted LP (the fixed
//                  glpk_interface.cpp:80-98) with its recovery map as
//                  trailing comment lines
//   --big-m M      artificial cost (default 1e6 * max(1, max |c_j|))
// The input file may be text or binary; binary is detected by its magic.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <string>
#include <vector>

#include "../../include/simplex.h"
#include "lp_io.h"
#include "mps_io.h"

using Clock = std::chrono::steady_clock;
using TimePoint = Clock::time_point;

static double seconds(const TimePoint& a, const TimePoint& b) { return std::chrono::duration<double>(b - a).count(); }

static void print_elapsed_time(const char* msg, double dur) {
    auto label = std::string(msg) + ": ";
    std::cout << std::setw(19) << label;
    std::cout << std::fixed << std::setprecision(2);
    std::cout << std::setw(6) << dur << '\n';
}

static void usage() {
    std::cerr << "usage: solver [--max-iter K] [--eps E] [--compat] [--device D] [--no-iter-lines] [--json]"
                 " [--threads T] [--write-bin F] [--write-text F] [--no-solve] [--ratio reference|guarded|harris]"
                 " [--piv-tol T] [--feas-tol T] [--refactor K] [--window W] [--pricing dantzig|devex|steepest] [--tableau]"
                 " [--mps [--big-m M]]"
                 " (<file> | --gen m n seed)\n";
}

int main(int argc, char* argv[]) {
    std::ios_base::sync_with_stdio(false);
    int64_t max_iter = INT64_MAX;
    double eps = 1e-7;
    int device = -1;
    bool iter_lines = true, json = false, gen = false, solve = true;
    int threads = 0;
    std::string write_bin, write_text;
    int64_t gm = 0, gn = 0;
    uint64_t gseed = 0;
    const char* path = nullptr;
    int ratio = -1, window = 0, pricing = SPX_PRICING_DANTZIG;
    double piv_tol = 1e-9, feas_tol = 1e-9, big_m = 0.0;
    int64_t refactor = 0;
    bool mps_in = false, tableau = false;
    for (int a = 1; a < argc; ++a) {
        const std::string s = argv[a];
        auto need = [&](int k) {
            if (a + k >= argc) {
                usage();
                std::exit(1);
            }
        };
        if (s == "--max-iter") { need(1); max_iter = std::strtoll(argv[++a], nullptr, 10); }
        else if (s == "--eps") { need(1); eps = std::strtod(argv[++a], nullptr); }
        else if (s == "--compat") { max_iter = 5; eps = 1e-4; }
        else if (s == "--device") { need(1); device = std::atoi(argv[++a]); }
        else if (s == "--no-iter-lines") iter_lines = false;
        else if (s == "--json") json = true;
        else if (s == "--threads") { need(1); threads = std::atoi(argv[++a]); }
        else if (s == "--write-bin") { need(1); write_bin = argv[++a]; }
        else if (s == "--write-text") { need(1); write_text = argv[++a]; }
        else if (s == "--no-solve") solve = false;
        else if (s == "--ratio") {
            need(1);
            const std::string r = argv[++a];
            ratio = r == "reference" ? SPX_RATIO_REFERENCE
                  : r == "guarded"   ? SPX_RATIO_GUARDED
                  : r == "harris"    ? SPX_RATIO_HARRIS
                                     : -2;
            if (ratio == -2) { usage(); return 1; }
        }
        else if (s == "--piv-tol") { need(1); piv_tol = std::strtod(argv[++a], nullptr); }
        else if (s == "--feas-tol") { need(1); feas_tol = std::strtod(argv[++a], nullptr); }
        else if (s == "--refactor") { need(1); refactor = std::strtoll(argv[++a], nullptr, 10); }
        else if (s == "--window") { need(1); window = std::atoi(argv[++a]); }
        else if (s == "--mps") mps_in = true;
        else if (s == "--tableau") tableau = true;
        else if (s == "--pricing") {
            need(1);
            const std::string r = argv[++a];
            pricing = r == "dantzig" ? SPX_PRICING_DANTZIG
                      : r == "devex"   ? SPX_PRICING_DEVEX
                      : r == "steepest" ? SPX_PRICING_STEEPEST
                                        : -1;
            if (pricing < 0) { usage(); return 1; }
        }
        else if (s == "--big-m") { need(1); big_m = std::strtod(argv[++a], nullptr); }
        else if (s == "--gen") {
            need(3);
            gen = true;
            gm = std::strtoll(argv[++a], nullptr, 10);
            gn = std::strtoll(argv[++a], nullptr, 10);
            gseed = std::strtoull(argv[++a], nullptr, 10);
        } else if (s == "-h" || s == "--help") { usage(); return 0; }
        else if (!path) path = argv[a];
        else { usage(); return 1; }
    }
    if (!path && !gen) {
        std::cerr << "Please, specify an input file.\n";
        return 1;
    }

    const TimePoint t_start = Clock::now();
    TimePoint t_host_alloc = t_start, t_read = t_start, t_solve = t_start;
    lpio::LP lp;
    mps::Problem pb;
    std::string err, trailer;
    if (mps_in && !gen) {
        t_host_alloc = t_read = Clock::now();
        if (mps::read_mps(path, pb, err, big_m) != 0) {
            std::cerr << err << "\n";
            return EXIT_FAILURE;
        }
        lp = std::move(pb.lp);
        trailer = mps::map_block(pb);
    } else if (!gen) {
        t_host_alloc = t_read = Clock::now();
        if (lpio::read_any(path, lp, err, threads) != 0) {
            std::cerr << err << "\n";
            return EXIT_FAILURE;
        }
    } else {
        lp.m = gm;
        lp.n = gn;
        t_host_alloc = t_read = Clock::now();
        if (!write_bin.empty() || !write_text.empty()) lpio::generate(gm, gn, gseed, lp);
    }
    if ((!write_bin.empty() && lpio::write_binary(write_bin, lp, err) != 0) ||
        (!write_text.empty() && lpio::write_text(write_text, lp, err, trailer) != 0)) {
        std::cerr << err << "\n";
        return EXIT_FAILURE;
    }
    if (!solve) return 0;
    const int64_t m = lp.m, n = lp.n;
    const bool device_gen = gen && lp.A.empty();
    std::vector<double> x_b((size_t)std::max<int64_t>(m, 1));
    std::vector<int64_t> b_ixs((size_t)std::max<int64_t>(m, 1));

    t_solve = Clock::now();
    spx_opts o;
    spx_default_opts(&o);
    o.eps = eps;
    o.device = device;
    o.ratio_test = ratio >= 0 ? ratio : (mps_in ? SPX_RATIO_GUARDED : SPX_RATIO_REFERENCE);
    o.piv_tol = piv_tol;
    o.feas_tol = feas_tol;
    o.refactor_every = (int32_t)refactor;
    o.window = window;
    o.pricing = pricing;
    if (tableau) o.flags |= SPX_FLAG_TABLEAU;
    spx_ctx* ctx = nullptr;
    const TimePoint t_alloc = Clock::now();
    int rc = device_gen ? spx_create_generated(&ctx, m, n, gseed, &o)
                        : spx_create(&ctx, m, n, lp.A.data(), lp.b.data(), lp.c.data(), &o);
    if (rc != SPX_OK) {
        std::cerr << "spx_create failed (" << rc << "): " << spx_last_error() << "\n";
        return EXIT_FAILURE;
    }
    const TimePoint t_init_end = Clock::now();
    double z = 0.0;
    int32_t status = 0;
    int64_t pivots = 0;
    rc = spx_solve(ctx, max_iter, &z, b_ixs.data(), x_b.data(), &status, &pivots);
    if (rc != SPX_OK) {
        std::cerr << "spx_solve failed (" << rc << "): " << spx_last_error() << "\n";
        spx_destroy(ctx);
        return EXIT_FAILURE;
    }
    const TimePoint t_loop_end = Clock::now();
    spx_destroy(ctx);
    const TimePoint t_dealloc_end = Clock::now();

    if (mps_in) {  // the reference's GLPK driver output (solver_glpk.cpp:27-38)
        pb.lp.m = m;
        pb.lp.n = n;
        std::vector<double> xb(x_b.begin(), x_b.begin() + m);
        std::vector<int64_t> bix(b_ixs.begin(), b_ixs.begin() + m);
        const double art = mps::max_artificial(pb, xb, bix);
        double bmax = 1.0;
        for (double v : lp.b) bmax = std::max(bmax, std::fabs(v));
        const bool feasible = art <= 1e-7 * bmax;
        const std::vector<double> xs = mps::recover_x(pb, xb, bix);
        const double zo = mps::objective(pb, xs);
        // GLPK status codes: GLP_OPT 5, GLP_NOFEAS 4, GLP_UNBND 6, GLP_UNDEF 1
        const int glp = status == SPX_STATUS_OPTIMUM_FOUND ? (feasible ? 5 : 4)
                        : status == SPX_STATUS_UNBOUNDED   ? 6
                                                           : 1;
        if (glp == 5) {
            for (size_t j = 0; j < xs.size(); ++j) std::cout << "x[" << j + 1 << "] = " << xs[j] << "\n";
            std::cout << "Optimal objective: " << zo << "\n";
        } else {
            std::cout << "Problem status: " << glp << "\n";
        }
        if (json) {
            std::cout << std::defaultfloat << std::setprecision(17);
            std::cout << "{\"status\": " << status << ", \"glp_status\": " << glp << ", \"z\": " << zo
                      << ", \"pivots\": " << pivots << ", \"m\": " << m << ", \"n\": " << n
                      << ", \"max_artificial\": " << art << ", \"x\": [";
            for (size_t j = 0; j < xs.size(); ++j) std::cout << (j ? ", " : "") << xs[j];
            std::cout << "]}\n";
        }
        return 0;
    }

    // "# Iteration k" once per loop pass (v4:287): pivots + the terminating pass
    const int64_t passes = (status == SPX_STATUS_MAX_ITER) ? pivots : pivots + 1;
    if (iter_lines)
        for (int64_t i = 1; i <= passes; ++i) std::cout << "# Iteration " << i << '\n';

    const TimePoint t_print = Clock::now();
    switch (status) {
        case SPX_STATUS_OPTIMUM_FOUND:
            std::cout << "Optimum found: " << z << '\n';
            for (int64_t i = 0; i < m; ++i) std::cout << "\tx_" << b_ixs[(size_t)i] << " = " << x_b[(size_t)i] << "\n";
            break;
        case SPX_STATUS_UNBOUNDED: std::cout << "Problem unbounded.\n"; break;
        case SPX_STATUS_THETA_OVERFLOW: std::cout << "Theta overflow.\n"; break;
        default: std::cout << "MAX_ITER exceeded.\n"; break;
    }
    std::cout << '\n';
    const TimePoint t_host_free = Clock::now();
    lp = lpio::LP();
    const TimePoint t_end = Clock::now();

    // timing table (v4:456-471).  The reference's y / x_b phases are fused into
    // the update kernel here, so the whole device loop is reported under p and
    // B_inv is 0 (per-kernel device times: bench.py / spx_kernel_times).
    print_elapsed_time("Total", seconds(t_start, t_end));
    std::cout << '\n';
    print_elapsed_time("y", 0.0);
    print_elapsed_time("p", seconds(t_init_end, t_loop_end));
    print_elapsed_time("B_inv", 0.0);
    print_elapsed_time("x_b", 0.0);
    std::cout << '\n';
    print_elapsed_time("Alloc", seconds(t_alloc, t_init_end));
    print_elapsed_time("Init", 0.0);
    print_elapsed_time("Dealloc", seconds(t_loop_end, t_dealloc_end));
    std::cout << '\n';
    print_elapsed_time("Host alloc", seconds(t_host_alloc, t_read));
    print_elapsed_time("Read file", seconds(t_read, t_solve));
    print_elapsed_time("Solve call", seconds(t_solve, t_print));
    print_elapsed_time("Print result", seconds(t_print, t_host_free));
    print_elapsed_time("Host free", seconds(t_host_free, t_end));

    if (json) {
        std::cout << std::defaultfloat << std::setprecision(17);
        std::cout << "{\"status\": " << status << ", \"z\": " << z << ", \"pivots\": " << pivots
                  << ", \"m\": " << m << ", \"n\": " << n
                  << ", \"solve_s\": " << seconds(t_init_end, t_loop_end) << "}\n";
    }
    return 0;
}
