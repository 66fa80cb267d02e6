// mps_io.h — MPS input for the ./solver CLI.
//
// The reference reads MPS only through GLPK: solver_glpk.cpp:15 (glp_read_mps,
// fixed deck) for its CPU baseline, and glpk_interface.cpp:6-98 (lp_from_mps
// + output_lp) to turn an MPS file into the solver's text format.  That
// converter is broken (glpk_interface.cpp:83 prints "m n" without a
// separator; :46-52,80-98 drop row senses and bounds and add no slacks).  This
// module replaces both: a self-contained MPS reader (fixed or free format:
// whitespace-separated fields, names without blanks) and a conversion to the
// solver's canonical form
//
//     max  c^T x   s.t.  A x = b,  x >= 0,  A = [structural | surplus | I_m],
//     b >= 0
//
// i.e. exactly the LP shape the reference's solve() assumes (slack basis
// A[:, n-m:] = I, b >= 0; v4:272-277).  Rows: L/G/E/N with RHS and RANGES;
// bounds: UP LO FX FR MI PL BV LI UI (integer markers and types are read as
// their LP relaxation).  Variables are shifted to x' = x - lo (or up - x, or
// split x+ - x- when free); finite upper bounds become rows; every row gets
// one identity column: a slack (cost 0) when its right-hand side is >= 0
// after sign normalisation, else a surplus column plus an artificial column
// with cost -M (big-M, one solve).  Minimisation is solved as max -c.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "lp_io.h"

namespace mps {

// How an original column maps onto canonical columns.
enum VarKind : int { kShift = 0, kMirror = 1, kSplit = 2, kFixed = 3 };
// kShift : x = shift + x'[plus]          (finite lower bound)
// kMirror: x = shift - x'[plus]          (lower -inf, finite upper)
// kSplit : x = x'[plus] - x'[minus]      (free)
// kFixed : x = shift                     (lo == up; no column)

struct Var {
    std::string name;
    int kind = kShift;
    int64_t plus = -1, minus = -1;
    double shift = 0.0;
    double cost = 0.0;  // original objective coefficient
};

struct Problem {
    std::string name;
    bool maximize = false;      // OBJSENSE MAX
    double obj_const = 0.0;     // constant of the original objective
    std::vector<Var> vars;      // original columns, file order
    std::vector<std::string> rows;  // original constraint rows, file order
    // canonical LP (lpio::LP: A column-major m x n, b, c)
    lpio::LP lp;
    std::vector<int64_t> artificial;  // canonical columns with cost -M
    double big_m = 0.0;
};

// Parse + convert.  big_m <= 0: M = 1e6 * max(1, max |c_j|).  Returns 0, or
// nonzero with err = "<file>:<line>: <message>".
int read_mps(const std::string& path, Problem& pb, std::string& err, double big_m = 0.0);

// Original x (file column order) from a canonical basic solution.
std::vector<double> recover_x(const Problem& pb, const std::vector<double>& x_b,
                              const std::vector<int64_t>& b_ixs);
// Original objective c^T x + constant.
double objective(const Problem& pb, const std::vector<double>& x);
// Largest artificial value in the basic solution (0 when none is basic).
double max_artificial(const Problem& pb, const std::vector<double>& x_b,
                      const std::vector<int64_t>& b_ixs);

// The trailing map block written after c by `--write-text` (ignored by the
// reference's reader, v4:94-104): lets a text file carry the recovery map.
std::string map_block(const Problem& pb);

}  // namespace mps
