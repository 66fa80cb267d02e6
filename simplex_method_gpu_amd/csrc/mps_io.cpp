// mps_io.cpp — MPS reader and canonical-form conversion (see mps_io.h).
#include "mps_io.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <limits>
#include <sstream>
#include <unordered_map>

namespace mps {
namespace {

constexpr double kInf = std::numeric_limits<double>::infinity();

struct RowDef {
    char type = 'L';  // 'L' 'G' 'E' 'N'
    double rhs = 0.0;
    double range = 0.0;
    bool has_range = false;
};

struct ColDef {
    std::string name;
    std::vector<std::pair<int64_t, double>> entries;  // (constraint row, value)
    double cost = 0.0;
    double lo = 0.0, up = kInf;
    bool lo_set = false;
};

bool to_double(const std::string& s, double* v) {
    char* e = nullptr;
    *v = std::strtod(s.c_str(), &e);
    return !s.empty() && e == s.c_str() + s.size();
}

std::vector<std::string> split(const std::string& line) {
    std::vector<std::string> t;
    std::istringstream is(line);
    std::string w;
    while (is >> w) t.push_back(w);
    return t;
}

std::string upper(std::string s) {
    for (char& ch : s) ch = (char)std::toupper((unsigned char)ch);
    return s;
}

// One row of the canonical LP under construction: sum coef x' (<= or =) rhs.
struct CRow {
    std::vector<std::pair<int64_t, double>> a;  // (canonical structural column, value)
    double rhs;
    bool eq;
};

}  // namespace

int read_mps(const std::string& path, Problem& pb, std::string& err, double big_m) {
    std::ifstream in(path);
    if (!in) {
        err = "Could not open " + path;
        return 1;
    }
    std::vector<RowDef> rows;  // constraint rows (N rows other than the objective are dropped)
    std::unordered_map<std::string, int64_t> row_ix;  // name -> constraint index, -1 objective, -2 free
    std::string obj_row;
    std::vector<ColDef> cols;
    std::unordered_map<std::string, int64_t> col_ix;
    std::string section, line;
    int64_t ln = 0;
    bool ended = false;
    auto bad = [&](const std::string& msg) {
        err = path + ":" + std::to_string(ln) + ": " + msg;
        return 1;
    };
    auto find_row = [&](const std::string& name, int64_t* r) -> bool {
        auto it = row_ix.find(name);
        if (it == row_ix.end()) return false;
        *r = it->second;
        return true;
    };
    while (std::getline(in, line)) {
        ++ln;
        if (!line.empty() && line.back() == '\r') line.pop_back();
        if (line.empty() || line[0] == '*') continue;
        std::vector<std::string> t = split(line);
        if (t.empty()) continue;
        if (line[0] != ' ' && line[0] != '\t') {  // section header
            section = upper(t[0]);
            if (section == "NAME") pb.name = t.size() > 1 ? t[1] : "";
            else if (section == "OBJSENSE" || section == "OBJSENCE") {
                if (t.size() > 1) pb.maximize = upper(t[1]).rfind("MAX", 0) == 0;
            } else if (section == "ENDATA") {
                ended = true;
                break;
            } else if (section != "ROWS" && section != "COLUMNS" && section != "RHS" && section != "RANGES" &&
                       section != "BOUNDS") {
                return bad("unknown section " + t[0]);
            }
            continue;
        }
        if (section == "OBJSENSE" || section == "OBJSENCE") {
            pb.maximize = upper(t[0]).rfind("MAX", 0) == 0;
        } else if (section == "ROWS") {
            if (t.size() < 2) return bad("ROWS entry needs a type and a name");
            const char ty = (char)std::toupper((unsigned char)t[0][0]);
            if (row_ix.count(t[1])) return bad("duplicate row " + t[1]);
            if (ty == 'N') {
                if (obj_row.empty()) {
                    obj_row = t[1];
                    row_ix[t[1]] = -1;
                } else {
                    row_ix[t[1]] = -2;  // further free rows are ignored (as GLPK's objective choice)
                }
            } else if (ty == 'L' || ty == 'G' || ty == 'E') {
                row_ix[t[1]] = (int64_t)rows.size();
                RowDef r;
                r.type = ty;
                rows.push_back(r);
                pb.rows.push_back(t[1]);
            } else {
                return bad("bad row type " + t[0]);
            }
        } else if (section == "COLUMNS") {
            if (t.size() >= 3 && upper(t[1]) == "'MARKER'") continue;  // INTORG / INTEND: LP relaxation
            if (t.size() != 3 && t.size() != 5) return bad("COLUMNS entry: column row value [row value]");
            auto it = col_ix.find(t[0]);
            int64_t j;
            if (it == col_ix.end()) {
                j = (int64_t)cols.size();
                col_ix[t[0]] = j;
                cols.emplace_back();
                cols.back().name = t[0];
            } else {
                j = it->second;
            }
            for (size_t k = 1; k + 1 < t.size(); k += 2) {
                int64_t r;
                double v;
                if (!find_row(t[k], &r)) return bad("unknown row " + t[k]);
                if (!to_double(t[k + 1], &v)) return bad("bad number " + t[k + 1]);
                if (r == -1) cols[(size_t)j].cost += v;
                else if (r >= 0) cols[(size_t)j].entries.emplace_back(r, v);
            }
        } else if (section == "RHS" || section == "RANGES") {
            // [set name] row value [row value]
            const size_t first = (t.size() % 2 == 1) ? 1 : 0;
            if (t.size() - first < 2) return bad(section + " entry: [set] row value [row value]");
            for (size_t k = first; k + 1 < t.size(); k += 2) {
                int64_t r;
                double v;
                if (!find_row(t[k], &r)) return bad("unknown row " + t[k]);
                if (!to_double(t[k + 1], &v)) return bad("bad number " + t[k + 1]);
                if (section == "RHS") {
                    if (r == -1) pb.obj_const = -v;  // RHS on the objective: minus the constant
                    else if (r >= 0) rows[(size_t)r].rhs = v;
                } else if (r >= 0) {
                    rows[(size_t)r].range = v;
                    rows[(size_t)r].has_range = true;
                }
            }
        } else if (section == "BOUNDS") {
            const std::string ty = upper(t[0]);
            const bool valued = !(ty == "FR" || ty == "MI" || ty == "PL" || ty == "BV");
            // type [set] column [value]
            const size_t want = valued ? 3 : 2;
            if (t.size() != want && t.size() != want + 1) return bad("BOUNDS entry: type [set] column [value]");
            const std::string& cname = t[t.size() == want + 1 ? 2 : 1];
            auto it = col_ix.find(cname);
            if (it == col_ix.end()) return bad("unknown column " + cname);
            ColDef& c = cols[(size_t)it->second];
            double v = 0.0;
            if (valued && !to_double(t.back(), &v)) return bad("bad number " + t.back());
            if (ty == "UP" || ty == "UI") {
                c.up = v;
                if (v < 0.0 && !c.lo_set) c.lo = -kInf;  // classic MPS: negative UP frees the lower bound
            } else if (ty == "LO" || ty == "LI") {
                c.lo = v;
                c.lo_set = true;
            } else if (ty == "FX") {
                c.lo = c.up = v;
                c.lo_set = true;
            } else if (ty == "FR") {
                c.lo = -kInf;
                c.up = kInf;
                c.lo_set = true;
            } else if (ty == "MI") {
                c.lo = -kInf;
                c.lo_set = true;
            } else if (ty == "PL") {
                c.up = kInf;
            } else if (ty == "BV") {
                c.lo = 0.0;
                c.up = 1.0;
                c.lo_set = true;
            } else {
                return bad("bad bound type " + t[0]);
            }
        } else {
            return bad("data outside a section");
        }
    }
    if (!ended) {
        err = path + ": missing ENDATA";
        return 1;
    }
    if (cols.empty()) {
        err = path + ": no columns";
        return 1;
    }
    for (const ColDef& c : cols)
        if (c.lo > c.up) {
            err = path + ": column " + c.name + " has lower bound > upper bound";
            return 1;
        }

    // ---- canonical form -------------------------------------------------
    // canonical structural columns x' and the map of the original columns
    int64_t nx = 0;
    pb.vars.clear();
    for (const ColDef& c : cols) {
        Var v;
        v.name = c.name;
        v.cost = c.cost;
        if (c.lo == c.up) {
            v.kind = kFixed;
            v.shift = c.lo;
        } else if (c.lo > -kInf) {
            v.kind = kShift;
            v.shift = c.lo;
            v.plus = nx++;
        } else if (c.up < kInf) {
            v.kind = kMirror;
            v.shift = c.up;
            v.plus = nx++;
        } else {
            v.kind = kSplit;
            v.plus = nx++;
            v.minus = nx++;
        }
        pb.vars.push_back(v);
    }
    // rows over x': every finite side of every constraint, then bound rows
    std::vector<std::vector<std::pair<int64_t, double>>> arow(rows.size());
    std::vector<double> delta(rows.size(), 0.0);  // sum a_ij shift_j
    for (size_t j = 0; j < cols.size(); ++j) {
        const Var& v = pb.vars[j];
        for (const auto& e : cols[j].entries) {
            const size_t r = (size_t)e.first;
            const double a = e.second;
            switch (v.kind) {
                case kFixed: delta[r] += a * v.shift; break;
                case kShift: delta[r] += a * v.shift; arow[r].emplace_back(v.plus, a); break;
                case kMirror: delta[r] += a * v.shift; arow[r].emplace_back(v.plus, -a); break;
                case kSplit: arow[r].emplace_back(v.plus, a); arow[r].emplace_back(v.minus, -a); break;
            }
        }
    }
    std::vector<CRow> crows;
    for (size_t r = 0; r < rows.size(); ++r) {
        const RowDef& d = rows[r];
        double lo = -kInf, up = kInf;
        if (d.type == 'L') up = d.rhs;
        else if (d.type == 'G') lo = d.rhs;
        else lo = up = d.rhs;
        if (d.has_range) {
            const double R = std::fabs(d.range);
            if (d.type == 'L') lo = d.rhs - R;
            else if (d.type == 'G') up = d.rhs + R;
            else if (d.range > 0) up = d.rhs + R;
            else lo = d.rhs - R;
        }
        lo -= delta[r];
        up -= delta[r];
        if (lo == up) {
            crows.push_back(CRow{arow[r], up, true});
            continue;
        }
        if (up < kInf) crows.push_back(CRow{arow[r], up, false});
        if (lo > -kInf) {  // a x >= lo  as  -a x <= -lo
            CRow cr{arow[r], -lo, false};
            for (auto& e : cr.a) e.second = -e.second;
            crows.push_back(cr);
        }
    }
    for (size_t j = 0; j < cols.size(); ++j) {  // finite upper bounds of shifted columns
        const Var& v = pb.vars[j];
        if (v.kind == kShift && cols[j].up < kInf)
            crows.push_back(CRow{{{v.plus, 1.0}}, cols[j].up - cols[j].lo, false});
    }
    if (crows.empty()) {  // no constraint: a dummy row 0 <= 1 keeps m >= 1
        crows.push_back(CRow{{}, 1.0, false});
    }
    // sign-normalise: rows with rhs < 0 flip; "<=" rows flipped become ">=":
    // surplus column + artificial; "=" rows get an artificial
    const int64_t m = (int64_t)crows.size();
    std::vector<int> needs_art((size_t)m, 0), surplus((size_t)m, 0);
    int64_t nsur = 0;
    for (int64_t i = 0; i < m; ++i) {
        CRow& cr = crows[(size_t)i];
        if (cr.rhs < 0.0) {
            cr.rhs = -cr.rhs;
            for (auto& e : cr.a) e.second = -e.second;
            if (!cr.eq) {
                surplus[(size_t)i] = 1;
                ++nsur;
            }
            needs_art[(size_t)i] = 1;
        } else if (cr.eq) {
            needs_art[(size_t)i] = 1;
        }
    }
    const int64_t n = nx + nsur + m;
    lpio::LP& lp = pb.lp;
    lp.m = m;
    lp.n = n;
    lp.A.assign((size_t)(m * n), 0.0);
    lp.b.assign((size_t)m, 0.0);
    lp.c.assign((size_t)n, 0.0);
    int64_t s = nx;
    for (int64_t i = 0; i < m; ++i) {
        const CRow& cr = crows[(size_t)i];
        for (const auto& e : cr.a) lp.A[(size_t)(i + e.first * m)] += e.second;
        if (surplus[(size_t)i]) lp.A[(size_t)(i + (s++) * m)] = -1.0;
        lp.A[(size_t)(i + (nx + nsur + i) * m)] = 1.0;
        lp.b[(size_t)i] = cr.rhs;
    }
    double cmax = 1.0;
    const double sense = pb.maximize ? 1.0 : -1.0;
    for (const Var& v : pb.vars) {
        const double cv = sense * v.cost;
        switch (v.kind) {
            case kShift: lp.c[(size_t)v.plus] += cv; break;
            case kMirror: lp.c[(size_t)v.plus] -= cv; break;
            case kSplit:
                lp.c[(size_t)v.plus] += cv;
                lp.c[(size_t)v.minus] -= cv;
                break;
            default: break;
        }
        cmax = std::max(cmax, std::fabs(v.cost));
    }
    pb.big_m = big_m > 0.0 ? big_m : 1e6 * cmax;
    pb.artificial.clear();
    for (int64_t i = 0; i < m; ++i)
        if (needs_art[(size_t)i]) {
            lp.c[(size_t)(nx + nsur + i)] = -pb.big_m;
            pb.artificial.push_back(nx + nsur + i);
        }
    return 0;
}

std::vector<double> recover_x(const Problem& pb, const std::vector<double>& x_b, const std::vector<int64_t>& b_ixs) {
    std::vector<double> xc((size_t)pb.lp.n, 0.0);
    for (size_t k = 0; k < b_ixs.size() && k < x_b.size(); ++k)
        if (b_ixs[k] >= 0 && b_ixs[k] < pb.lp.n) xc[(size_t)b_ixs[k]] = x_b[k];
    std::vector<double> x;
    x.reserve(pb.vars.size());
    for (const Var& v : pb.vars) {
        switch (v.kind) {
            case kFixed: x.push_back(v.shift); break;
            case kShift: x.push_back(v.shift + xc[(size_t)v.plus]); break;
            case kMirror: x.push_back(v.shift - xc[(size_t)v.plus]); break;
            default: x.push_back(xc[(size_t)v.plus] - xc[(size_t)v.minus]); break;
        }
    }
    return x;
}

double objective(const Problem& pb, const std::vector<double>& x) {
    double z = pb.obj_const;
    for (size_t j = 0; j < pb.vars.size() && j < x.size(); ++j) z += pb.vars[j].cost * x[j];
    return z;
}

double max_artificial(const Problem& pb, const std::vector<double>& x_b, const std::vector<int64_t>& b_ixs) {
    std::vector<char> art((size_t)pb.lp.n, 0);
    for (int64_t j : pb.artificial) art[(size_t)j] = 1;
    double mx = 0.0;
    for (size_t k = 0; k < b_ixs.size() && k < x_b.size(); ++k)
        if (b_ixs[k] >= 0 && b_ixs[k] < pb.lp.n && art[(size_t)b_ixs[k]]) mx = std::max(mx, x_b[k]);
    return mx;
}

std::string map_block(const Problem& pb) {
    std::ostringstream os;
    os.precision(17);
    os << "# spx-mps-map v1 name " << (pb.name.empty() ? "-" : pb.name) << "\n";
    os << "# sense " << (pb.maximize ? "max" : "min") << " const " << pb.obj_const << " big_m " << pb.big_m << "\n";
    for (size_t j = 0; j < pb.vars.size(); ++j) {
        const Var& v = pb.vars[j];
        os << "# var " << j << " " << v.name << " " << v.kind << " " << v.plus << " " << v.minus << " " << v.shift
           << " " << v.cost << "\n";
    }
    os << "# artificial";
    for (int64_t a : pb.artificial) os << " " << a;
    os << "\n";
    return os.str();
}

}  // namespace mps
