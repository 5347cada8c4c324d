// brhip_batch -- the reference's file-driven entry point batch_reactor(input_file, lib_dir;
// gaschem, surfchem) (src/BatchReactor.jl:67-70,:152-217) as a C++ program on libbrhip.so's C-ABI
// only: br_read_batch_xml, br_mech_parse / br_mech_create, br_integrate_traced. It is what the Julia
// module (julia/BatchReactorHIP.jl) does, line for line, and shows that the engine runs from the
// mechanism library files without Python. Writes gas_profile.{dat,csv} and surface_covg.{dat,csv}
// next to the input (save_data, :168-180,:383-402) and prints the retcode symbol.
//
//   brhip_batch <batch.xml> <lib_dir> [--gas] [--surf] [--device D]
//   brhip_batch --fmt < numbers      (prints Julia's string(::Float64) of each; tests)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/brhip.h"

namespace {

constexpr double R_GAS = 8.31446261815324;   // RxnHelperUtils.R (src/BatchReactor.jl:338)

// Julia's string(::Float64): shortest round-trip digits; plain notation for decimal exponents
// -4 <= e <= 5, d.ddde<exp> otherwise; always a fractional part (the golden CSV's format)
std::string julia_string(double x) {
    if (std::isnan(x)) return "NaN";
    if (std::isinf(x)) return x > 0 ? "Inf" : "-Inf";
    if (x == 0.0) return std::signbit(x) ? "-0.0" : "0.0";
    char buf[64];
    int prec = 1;
    for (; prec <= 17; ++prec) {   // shortest %.{prec-1}e that reads back as x
        std::snprintf(buf, sizeof(buf), "%.*e", prec - 1, x);
        if (std::strtod(buf, nullptr) == x) break;
    }
    // buf = [-]d.ddde[+-]XX -> sign, digits, exponent
    std::string s(buf);
    std::string sign;
    if (s[0] == '-') { sign = "-"; s = s.substr(1); }
    const size_t epos = s.find('e');
    const int e10 = std::atoi(s.c_str() + epos + 1);
    std::string digits;
    for (size_t i = 0; i < epos; ++i) if (s[i] != '.') digits += s[i];
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    if (e10 >= -4 && e10 <= 5) {
        std::string ip, fp;
        if (e10 >= 0) {
            ip = digits.substr(0, std::min(digits.size(), (size_t)e10 + 1));
            while ((int)ip.size() < e10 + 1) ip += '0';
            fp = digits.size() > (size_t)e10 + 1 ? digits.substr(e10 + 1) : "";
        } else {
            ip = "0";
            fp = std::string(-e10 - 1, '0') + digits;
        }
        return sign + ip + "." + (fp.empty() ? "0" : fp);
    }
    return sign + digits.substr(0, 1) + "." + (digits.size() > 1 ? digits.substr(1) : "0") + "e" + std::to_string(e10);
}

// numpy's sum of a contiguous double array (pairwise: 8 partial sums per block of <= 128), so the
// rows match the Python host's files bit for bit (the reference's Julia `sum` blocks differently;
// either way the difference is rounding)
double np_sum(const double* a, size_t n) {
    if (n < 8) {
        double r = 0.0;
        for (size_t i = 0; i < n; ++i) r += a[i];
        return r;
    }
    if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        size_t i = 8;
        for (; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    size_t n2 = n / 2;
    n2 -= n2 % 8;
    return np_sum(a, n2) + np_sum(a + n2, n - n2);
}

int check(int rc, const char* what) {
    if (rc) {
        std::fprintf(stderr, "%s: error %d: %s\n", what, rc, br_last_error());
        std::exit(2);
    }
    return rc;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc == 2 && !std::strcmp(argv[1], "--fmt")) {   // test hook: Julia string() of stdin's numbers
        char tok[128];
        while (std::scanf("%127s", tok) == 1) std::printf("%s\n", julia_string(std::strtod(tok, nullptr)).c_str());
        return 0;
    }
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <batch.xml> <lib_dir> [--gas] [--surf] [--device D]\n", argv[0]);
        return 2;
    }
    const std::string input = argv[1], libdir = argv[2];
    bool gas = false, surf = false;
    int device = 0;
    for (int i = 3; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--gas")) gas = true;
        else if (!std::strcmp(argv[i], "--surf")) surf = true;
        else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
    }
    auto path = [&](const char* f) { return libdir + "/" + f; };
    br_batch_input in;
    check(br_read_batch_xml(input.c_str(), &in), "br_read_batch_xml");
    br_host_mech* hm = nullptr;
    const std::string gm = gas ? path(in.gas_mech) : "", sm = surf ? path(in.surface_mech) : "";
    check(br_mech_parse(gm.c_str(), path("therm.dat").c_str(), sm.c_str(), gas ? "" : in.gasphase, BR_CONV_REFERENCE, &hm),
          "br_mech_parse");
    br_mech_desc d;
    check(br_host_mech_desc(hm, &d), "br_host_mech_desc");
    br_mech* m = nullptr;
    check(br_mech_create(&d, device, &m), "br_mech_create");
    const int ng = d.ng, ns = d.ns, n = ng + ns;
    std::vector<std::string> names(n);
    for (int i = 0; i < n; ++i) {
        char b[64];
        check(br_host_mech_species(hm, i, b, sizeof(b)), "br_host_mech_species");
        names[i] = b;
    }
    std::vector<double> molwt(d.molwt, d.molwt + ng), theta0(ns);
    check(br_host_mech_theta0(hm, theta0.data()), "br_host_mech_theta0");

    // get_solution_vector (:224-232): composition by name, rho0 = p Mbar / (R T), u = [rho Y ; theta0]
    std::vector<double> v(ng, 0.0);
    for (int c = 0; c < in.ncomp; ++c)
        for (int k = 0; k < ng; ++k)
            if (names[k] == in.comp_names[c]) v[k] = in.comp_values[c];
    if (in.comp_is_mass) {
        for (int k = 0; k < ng; ++k) v[k] /= molwt[k];
        const double s = np_sum(v.data(), ng);
        for (int k = 0; k < ng; ++k) v[k] /= s;
    }
    std::vector<double> xm(ng);
    for (int k = 0; k < ng; ++k) xm[k] = v[k] * molwt[k];
    const double Mb = np_sum(xm.data(), ng);
    const double rho = in.p * Mb / (R_GAS * in.T);
    std::vector<double> u0(n);
    for (int k = 0; k < ng; ++k) u0[k] = (v[k] * molwt[k] / Mb) * rho;
    for (int k = 0; k < ns; ++k) u0[ng + k] = theta0[k];

    // solve(...; callback = FunctionCallingCallback(save_data)) (:208-210): the traced integration;
    // the trace starts at 4096 rows and a longer run is repeated once with its exact step count
    br_opts o;
    std::memset(&o, 0, sizeof(o));
    o.rtol = 1e-6; o.atol = 1e-10; o.max_steps = 100000; o.device = device;
    int oh = 0;
    for (int k = 0; k < ng; ++k) if (names[k] == "OH") oh = k + 1;
    o.ignition_species = oh;
    int cap = 4096, nst = 0;
    std::vector<double> u, trace;
    br_stats st;
    for (int pass = 0; pass < 2; ++pass) {
        o.trace_cap = cap;
        u = u0;
        trace.assign((size_t)(cap + 1) * (2 * n + 4), 0.0);
        check(br_integrate_traced(m, 1, &in.T, &in.Asv, u.data(), &in.time, &o, &st, trace.data()), "br_integrate_traced");
        nst = (int)st.nsteps;
        if (nst <= cap) break;
        cap = nst;
    }

    // save_data rows: t, T, p, rho, x_k (gas_profile) and t, T, theta_k (surface_covg)
    std::string folder = input.substr(0, input.find_last_of('/') == std::string::npos ? 0 : input.find_last_of('/') + 1);
    if (folder.empty()) folder = "./";
    FILE* g_dat = std::fopen((folder + "gas_profile.dat").c_str(), "w");
    FILE* s_dat = std::fopen((folder + "surface_covg.dat").c_str(), "w");
    FILE* g_csv = std::fopen((folder + "gas_profile.csv").c_str(), "w");
    FILE* s_csv = std::fopen((folder + "surface_covg.csv").c_str(), "w");
    if (!g_dat || !s_dat || !g_csv || !s_csv) { std::fprintf(stderr, "cannot open output files in %s\n", folder.c_str()); return 2; }
    std::vector<std::string> gh = {"t", "T", "p", "rho"}, shh = {"t", "T"};
    for (int k = 0; k < ng; ++k) gh.push_back(names[k]);
    for (int k = 0; k < ns; ++k) shh.push_back(names[ng + k]);
    auto write_header = [&](FILE* dat, FILE* csv, const std::vector<std::string>& h) {
        for (const auto& x : h) std::fprintf(dat, "%10s\t", x.c_str());
        std::fprintf(dat, "\n");
        for (size_t i = 0; i < h.size(); ++i) std::fprintf(csv, "%s%s", i ? "," : "", h[i].c_str());
        std::fprintf(csv, "\n");
    };
    auto write_row = [&](FILE* dat, FILE* csv, const std::vector<double>& r) {
        for (double x : r) std::fprintf(dat, "%.4e\t", x);
        std::fprintf(dat, "\n");
        for (size_t i = 0; i < r.size(); ++i) std::fprintf(csv, "%s%s", i ? "," : "", julia_string(r[i]).c_str());
        std::fprintf(csv, "\n");
    };
    write_header(g_dat, g_csv, gh);
    if (surf) write_header(s_dat, s_csv, shh);
    for (int k = 0; k <= nst; ++k) {
        const double* row = &trace[(size_t)k * (2 * n + 4)];
        const double* uk = row + 4;
        const double* yk = row + 4 + n;
        const double su = np_sum(uk, ng), sy = np_sum(yk, ng);   // state_to_molefrac (:142-144)
        std::vector<double> gr = {row[0], in.T, row[3], su}, x(ng);
        for (int j = 0; j < ng; ++j) x[j] = (yk[j] / sy) / molwt[j];
        const double sx = np_sum(x.data(), ng);
        for (int j = 0; j < ng; ++j) gr.push_back(x[j] / sx);
        write_row(g_dat, g_csv, gr);
        if (surf) {
            std::vector<double> sr = {row[0], in.T};
            for (int j = 0; j < ns; ++j) sr.push_back(yk[ng + j]);
            write_row(s_dat, s_csv, sr);
        }
    }
    std::fclose(g_dat); std::fclose(s_dat); std::fclose(g_csv); std::fclose(s_csv);
    br_mech_destroy(m);
    br_host_mech_free(hm);
    std::printf("%s\n", st.status == 0 ? "Success" : "Failure");
    return st.status == 0 ? 0 : 1;
}
