/*
 * oracle.c -- CPU restatement of BatchReactor.jl's hot path. TEST INFRASTRUCTURE ONLY:
 * loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * checker / CPU baseline; never by the product (libbrhip.so). See oracle.h for the map
 * from each function to the reference file:line it follows.
 *
 * Plain C99 (+ optional OpenMP for the ensemble CPU baseline). Everything is fp64.
 */
#include "oracle.h"
#include <ctype.h>
#include <float.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MAXSP 160
#define NL 32
#define MAXE 6 /* expanded reactant/product entries per reaction */

static const double R_GAS = 8.31446261815324; /* RxnHelperUtils.R (src/Constants.jl:1 same value) */
static const double CAL2J = 4.184;

static __thread char g_err[512];
const char* orc_errmsg(void) { return g_err; }
static void seterr(const char* fmt, ...) {
    va_list ap; va_start(ap, fmt); vsnprintf(g_err, sizeof g_err, fmt, ap); va_end(ap);
}

/* ----------------------------------------------------------------------------------- */
/* mechanism data                                                                      */
/* ----------------------------------------------------------------------------------- */
typedef struct {
    char name[NL];
    double tlo, tmid, thi, hi[7], lo[7];
    int nel; char el[6][4]; double cnt[6];
} thermo_t;

typedef struct {
    int nf, nr, f[MAXE], r[MAXE];
    int rev, tb, troe, has_t2, dnu;
    double A, b, EoR;          /* SI pre-exponential, beta, Ea/R [K] (kinf for falloff) */
    double A0, b0, E0oR;       /* low-pressure limit (SI) */
    double ta, t3, t1, t2;
    double* eff;               /* [ng], NULL if tb==0 */
    double fmul, rmul;         /* per-reaction multipliers on the forward / reverse terms
                                  (1.0; convention-fitting hook for tests, orc_set_rxn_mult) */
} grxn_t;

typedef struct {
    int nf, np, f[MAXE], p[MAXE];   /* combined index: gas 0..ng-1, surface ng.. */
    int stick, stick_gas;
    double A, b, Ea;                /* SI (arrhenius) or s0 (stick); Ea [J/mol] */
    int ncov, cov_sp[8]; double cov_eps[8];  /* eps [J/mol], cov_sp combined index */
} srxn_t;

struct orc_mech {
    int ng, ns, nrg, nrs, conv;
    double p_std;
    char names[MAXSP][NL];
    double M[MAXSP];
    thermo_t th[MAXSP];
    grxn_t* gr;
    srxn_t* sr;
    double site_density;          /* mol/cm2 */
    double sigma[MAXSP];          /* per surface species */
    double th0[MAXSP];
};

int orc_ng(const orc_mech* m) { return m->ng; }
int orc_ns(const orc_mech* m) { return m->ns; }
int orc_nrg(const orc_mech* m) { return m->nrg; }
int orc_nrs(const orc_mech* m) { return m->nrs; }
const char* orc_species_name(const orc_mech* m, int k) { return m->names[k]; }
double orc_molwt(const orc_mech* m, int k) { return m->M[k]; }
double orc_site_density(const orc_mech* m) { return m->site_density; }
void orc_initial_coverage(const orc_mech* m, double* th) { for (int i = 0; i < m->ns; ++i) th[i] = m->th0[i]; }
void orc_set_conv(orc_mech* m, int conv) { m->conv = conv; }
void orc_set_rxn_mult(orc_mech* m, int i, double fmul, double rmul) {
    if (i >= 0 && i < m->nrg) { m->gr[i].fmul = fmul; m->gr[i].rmul = rmul; }
}

/* atomic weights [g/mol]. H/C/O/N fitted to the golden: they reproduce rho0 of
 * test/batch_gas_and_surf/gas_profile.csv row 1 bit-exactly and p(t) on every golden row
 * to 3.5e-11 (IdealGas's table is not vendored). */
static double atomic_weight(const char* e) {
    static const struct { const char* s; double w; } tab[] = {
        {"H", 1.0078}, {"C", 12.0107}, {"O", 15.99977}, {"N", 14.00643}, {"AR", 39.948},
        {"HE", 4.002602}, {"NE", 20.1797}, {"S", 32.065}, {"CL", 35.453}, {"F", 18.9984},
        {"E", 5.48579909e-4}};
    for (size_t i = 0; i < sizeof tab / sizeof tab[0]; ++i)
        if (!strcmp(tab[i].s, e)) return tab[i].w;
    return -1.0;
}

/* ----------------------------------------------------------------------------------- */
/* small string helpers                                                                */
/* ----------------------------------------------------------------------------------- */
static void upcase(char* s) { for (; *s; ++s) *s = (char)toupper((unsigned char)*s); }
static char* trim(char* s) {
    while (*s && isspace((unsigned char)*s)) ++s;
    char* e = s + strlen(s);
    while (e > s && isspace((unsigned char)e[-1])) *--e = 0;
    return s;
}
static char* read_file(const char* path) {
    FILE* f = fopen(path, "rb");
    if (!f) { seterr("cannot open %s", path); return NULL; }
    fseek(f, 0, SEEK_END); long n = ftell(f); fseek(f, 0, SEEK_SET);
    char* b = (char*)malloc((size_t)n + 1);
    if (fread(b, 1, (size_t)n, f) != (size_t)n) { fclose(f); free(b); seterr("read %s", path); return NULL; }
    b[n] = 0; fclose(f);
    return b;
}
static int find_species(const orc_mech* m, const char* nm, int lo, int hi) {
    for (int k = lo; k < hi; ++k) if (!strcmp(m->names[k], nm)) return k;
    return -1;
}

/* ----------------------------------------------------------------------------------- */
/* NASA-7 therm.dat (IdealGas.create_thermo, src/BatchReactor.jl:265)                  */
/* ----------------------------------------------------------------------------------- */
static double fnum(const char* line, int col, int w) {
    char buf[32]; int L = (int)strlen(line);
    if (col >= L) return 0.0;
    int n = w; if (col + n > L) n = L - col;
    memcpy(buf, line + col, (size_t)n); buf[n] = 0;
    for (char* c = buf; *c; ++c) if (*c == 'D' || *c == 'd') *c = 'E';
    return atof(buf);
}
static int load_thermo(const char* path, thermo_t** out) {
    char* txt = read_file(path);
    if (!txt) return -1;
    int cap = 512, n = 0;
    thermo_t* t = (thermo_t*)calloc((size_t)cap, sizeof *t);
    char* lines[8192]; int nl = 0;
    for (char* s = strtok(txt, "\n"); s && nl < 8192; s = strtok(NULL, "\n")) {
        size_t L = strlen(s); if (L && s[L - 1] == '\r') s[L - 1] = 0;
        lines[nl++] = s;
    }
    for (int i = 0; i + 3 < nl; ++i) {
        char* l = lines[i];
        int L = (int)strlen(l);
        if (L < 80 || l[79] != '1' || l[0] == '!') continue;
        if (strlen(lines[i + 1]) < 79 || lines[i + 1][79] != '2') continue;
        thermo_t* e = &t[n];
        memset(e, 0, sizeof *e);
        sscanf(l, "%31s", e->name); upcase(e->name);
        for (int k = 0; k < 4; ++k) {
            char sym[4] = {0}; memcpy(sym, l + 24 + 5 * k, 2);
            char* s = trim(sym); upcase(s);
            double c = fnum(l, 26 + 5 * k, 3);
            if (*s && c != 0.0 && strcmp(s, "0")) { strcpy(e->el[e->nel], s); e->cnt[e->nel++] = c; }
        }
        e->tlo = fnum(l, 45, 10); e->thi = fnum(l, 55, 10); e->tmid = fnum(l, 65, 8);
        if (e->tmid == 0.0) e->tmid = 1000.0;
        double a[15];
        for (int k = 0; k < 5; ++k) a[k] = fnum(lines[i + 1], 15 * k, 15);
        for (int k = 0; k < 5; ++k) a[5 + k] = fnum(lines[i + 2], 15 * k, 15);
        for (int k = 0; k < 4; ++k) a[10 + k] = fnum(lines[i + 3], 15 * k, 15);
        for (int k = 0; k < 7; ++k) { e->hi[k] = a[k]; e->lo[k] = a[7 + k]; }
        if (++n == cap) { cap *= 2; t = (thermo_t*)realloc(t, (size_t)cap * sizeof *t); }
        i += 3;
    }
    free(txt);
    *out = t;
    return n;
}

static int attach_thermo(orc_mech* m, thermo_t* tab, int nt) {
    for (int k = 0; k < m->ng; ++k) {
        int found = 0;
        for (int i = 0; i < nt; ++i) if (!strcmp(tab[i].name, m->names[k])) {
            m->th[k] = tab[i]; found = 1;
            double w = 0;
            for (int e = 0; e < tab[i].nel; ++e) {
                double aw = atomic_weight(tab[i].el[e]);
                if (aw < 0) { seterr("unknown element %s", tab[i].el[e]); return -1; }
                w += tab[i].cnt[e] * aw;
            }
            m->M[k] = w * 1e-3;
            break;
        }
        if (!found) { seterr("species %s not in therm.dat", m->names[k]); return -1; }
    }
    return 0;
}

/* ----------------------------------------------------------------------------------- */
/* CHEMKIN-II gas mechanism (GasphaseReactions.compile_gaschemistry, :254)              */
/* ----------------------------------------------------------------------------------- */
static int parse_side(orc_mech* m, char* side, int* idx, int* ne, int* has_m) {
    /* terms separated by '+'; 'M' = third body; leading integer = stoichiometric coef */
    *ne = 0;
    char* save = NULL;
    for (char* tok = strtok_r(side, "+", &save); tok; tok = strtok_r(NULL, "+", &save)) {
        char* t = trim(tok);
        if (!*t) continue;
        int coef = 1;
        if (isdigit((unsigned char)t[0])) {
            int c = 0; while (isdigit((unsigned char)*t)) c = c * 10 + (*t++ - '0');
            coef = c;
        }
        if (!strcmp(t, "M")) { *has_m = 1; continue; }
        int k = find_species(m, t, 0, m->ng);
        if (k < 0) { seterr("unknown species '%s' in reaction", t); return -1; }
        for (int c = 0; c < coef; ++c) { if (*ne >= MAXE) { seterr("too many entries"); return -1; } idx[(*ne)++] = k; }
    }
    return 0;
}

static int load_chemkin(orc_mech* m, const char* path) {
    char* txt = read_file(path);
    if (!txt) return -1;
    enum { NONE, ELEM, SPEC, THERMO, REAC } sec = NONE;
    double efac = CAL2J / R_GAS; /* Ea units -> K */
    int cap = 64; m->gr = (grxn_t*)calloc((size_t)cap, sizeof(grxn_t)); m->nrg = 0;
    char* save = NULL;
    for (char* raw = strtok_r(txt, "\n", &save); raw; raw = strtok_r(NULL, "\n", &save)) {
        char* bang = strchr(raw, '!'); if (bang) *bang = 0;
        char line[1024]; snprintf(line, sizeof line, "%s", raw);
        upcase(line);
        char* l = trim(line);
        if (!*l) continue;
        char first[64] = {0}; sscanf(l, "%63s", first);
        if (!strncmp(first, "ELEM", 4)) { sec = ELEM; continue; }
        if (!strncmp(first, "SPEC", 4)) { sec = SPEC; l += strlen(first); if (!*trim(l)) continue; }
        if (!strncmp(first, "THERMO", 6)) { sec = THERMO; continue; }
        if (!strncmp(first, "REAC", 4)) {
            sec = REAC;
            if (strstr(l, "KCAL/MOLE")) efac = 1000.0 * CAL2J / R_GAS;
            else if (strstr(l, "KJOULES/MOLE")) efac = 1000.0 / R_GAS;
            else if (strstr(l, "JOULES/MOLE")) efac = 1.0 / R_GAS;
            else if (strstr(l, "KELVINS")) efac = 1.0;
            continue;
        }
        if (!strcmp(first, "END")) { sec = NONE; continue; }
        if (sec == SPEC) {
            char* s2 = NULL;
            for (char* t = strtok_r(l, " \t", &s2); t; t = strtok_r(NULL, " \t", &s2)) {
                if (!strcmp(t, "END")) { sec = NONE; break; }
                if (find_species(m, t, 0, m->ng) < 0) snprintf(m->names[m->ng++], NL, "%s", t);
            }
            continue;
        }
        if (sec != REAC) continue;
        if (strchr(l, '=')) {
            /* new reaction: last three tokens are A, beta, E */
            char* toks[64]; int nt = 0; char* s2 = NULL;
            char work[1024]; snprintf(work, sizeof work, "%s", l);
            for (char* t = strtok_r(work, " \t", &s2); t && nt < 64; t = strtok_r(NULL, " \t", &s2)) toks[nt++] = t;
            if (nt < 4) { seterr("bad reaction line: %s", l); return -1; }
            double A = atof(toks[nt - 3]), b = atof(toks[nt - 2]), E = atof(toks[nt - 1]);
            char eq[512] = {0};
            for (int i = 0; i < nt - 3; ++i) strncat(eq, toks[i], sizeof eq - strlen(eq) - 1);
            if (m->nrg == cap) { cap *= 2; m->gr = (grxn_t*)realloc(m->gr, (size_t)cap * sizeof(grxn_t)); }
            grxn_t* r = &m->gr[m->nrg]; memset(r, 0, sizeof *r);
            r->fmul = r->rmul = 1.0;
            /* falloff marker "(+M)" */
            char* pm;
            int falloff = 0;
            while ((pm = strstr(eq, "(+M)"))) { falloff = 1; memmove(pm, pm + 4, strlen(pm + 4) + 1); }
            char *lhs = eq, *rhs;
            if ((rhs = strstr(eq, "<=>"))) { *rhs = 0; rhs += 3; r->rev = 1; }
            else if ((rhs = strstr(eq, "=>"))) { *rhs = 0; rhs += 2; r->rev = 0; }
            else { rhs = strchr(eq, '='); *rhs = 0; rhs += 1; r->rev = 1; }
            int hm1 = 0, hm2 = 0;
            if (parse_side(m, lhs, r->f, &r->nf, &hm1) || parse_side(m, rhs, r->r, &r->nr, &hm2)) return -1;
            r->tb = falloff ? 2 : ((hm1 || hm2) ? 1 : 0);
            r->dnu = r->nr - r->nf;
            int order = r->nf + (r->tb == 1 ? 1 : 0);
            r->A = A * pow(1e-6, order - 1);
            r->b = b; r->EoR = E * efac;
            if (r->tb) {
                r->eff = (double*)malloc((size_t)m->ng * sizeof(double));
                for (int k = 0; k < m->ng; ++k) r->eff[k] = 1.0;
            }
            m->nrg++;
            continue;
        }
        /* auxiliary line for the last reaction */
        if (m->nrg == 0) continue;
        grxn_t* r = &m->gr[m->nrg - 1];
        if (!strncmp(first, "DUP", 3)) continue;
        /* tokenise on '/' */
        char work[1024]; snprintf(work, sizeof work, "%s", l);
        char* parts[64]; int np = 0;
        char* p = work;
        while (np < 64) {
            char* sl = strchr(p, '/');
            if (!sl) { if (*trim(p)) parts[np++] = trim(p); break; }
            *sl = 0; parts[np++] = trim(p); p = sl + 1;
        }
        for (int i = 0; i + 1 < np; i += 2) {
            char* key = parts[i]; char* val = parts[i + 1];
            if (!*key) { --i; continue; }
            if (!strcmp(key, "LOW")) {
                double a0, b0, e0; sscanf(val, "%lf %lf %lf", &a0, &b0, &e0);
                r->A0 = a0 * pow(1e-6, r->nf); r->b0 = b0; r->E0oR = e0 * efac;
            } else if (!strcmp(key, "TROE")) {
                double v[4] = {0}; int nv = sscanf(val, "%lf %lf %lf %lf", &v[0], &v[1], &v[2], &v[3]);
                r->troe = 1; r->ta = v[0]; r->t3 = v[1]; r->t1 = v[2]; r->t2 = v[3]; r->has_t2 = (nv == 4);
            } else if (!strcmp(key, "REV") || !strcmp(key, "SRI") || !strcmp(key, "PLOG") || !strcmp(key, "FORD")) {
                seterr("unsupported keyword %s", key); return -1;
            } else {
                int k = find_species(m, key, 0, m->ng);
                if (k >= 0 && r->eff) r->eff[k] = atof(val);
            }
        }
    }
    free(txt);
    return 0;
}

/* ----------------------------------------------------------------------------------- */
/* surface mechanism XML (SurfaceReactions.compile_mech, :287; ch4ni.xml)               */
/* ----------------------------------------------------------------------------------- */
static char* tag_body(char* s, const char* tag, char** after, char* attrs, size_t attrn) {
    char open[64]; snprintf(open, sizeof open, "<%s", tag);
    char* p = s;
    for (;;) {
        p = strstr(p, open);
        if (!p) return NULL;
        char c = p[strlen(open)];
        if (c == '>' || isspace((unsigned char)c)) break;
        p += 1;
    }
    char* gt = strchr(p, '>');
    if (!gt) return NULL;
    if (attrs) {
        size_t n = (size_t)(gt - (p + strlen(open)));
        if (n >= attrn) n = attrn - 1;
        memcpy(attrs, p + strlen(open), n); attrs[n] = 0;
    }
    char close[64]; snprintf(close, sizeof close, "</%s>", tag);
    char* e = strstr(gt + 1, close);
    if (!e) return NULL;
    *e = 0;
    if (after) *after = e + strlen(close);
    return gt + 1;
}
static int surf_index(const orc_mech* m, const char* nm) {
    int k = find_species(m, nm, m->ng, m->ng + m->ns);
    if (k >= 0) return k;
    return find_species(m, nm, 0, m->ng);
}
static int parse_surf_side(orc_mech* m, char* side, int* idx, int* ne) {
    *ne = 0; char* save = NULL;
    for (char* t = strtok_r(side, "+", &save); t; t = strtok_r(NULL, "+", &save)) {
        char* s = trim(t); if (!*s) continue;
        int coef = 1;
        if (isdigit((unsigned char)s[0])) { coef = 0; while (isdigit((unsigned char)*s)) coef = coef * 10 + (*s++ - '0'); s = trim(s); }
        int k = surf_index(m, s);
        if (k < 0) { seterr("unknown surface-reaction species '%s'", s); return -1; }
        for (int c = 0; c < coef; ++c) idx[(*ne)++] = k;
    }
    return 0;
}
static int load_surface(orc_mech* m, const char* path) {
    char* txt = read_file(path);
    if (!txt) return -1;
    /* strip comments */
    for (char* c; (c = strstr(txt, "<!--"));) {
        char* e = strstr(c, "-->");
        if (!e) { *c = 0; break; }
        memmove(c, e + 3, strlen(e + 3) + 1);
    }
    upcase(txt);
    char root_attr[256] = {0};
    char* rest = NULL;
    /* unit attribute on the root element */
    double efac = 1000.0; /* kJ/mol default for ch4ni.xml */
    {
        char* r0 = strstr(txt, "<SURFACE_CHEMISRTY");
        if (!r0) r0 = strstr(txt, "<SURFACE_CHEMISTRY");
        if (r0) { char* gt = strchr(r0, '>'); size_t n = (size_t)(gt - r0); if (n > 255) n = 255; memcpy(root_attr, r0, n); }
        if (strstr(root_attr, "UNIT=\"J/MOL\"")) efac = 1.0;
        if (strstr(root_attr, "UNIT=\"KCAL/MOL\"")) efac = 4184.0;
        if (strstr(root_attr, "UNIT=\"CAL/MOL\"")) efac = CAL2J;
    }
    char* work = strdup(txt);
    char* sp = tag_body(work, "SPECIES", &rest, NULL, 0);
    if (!sp) { seterr("no <species> in %s", path); return -1; }
    m->ns = 0;
    char* s2 = NULL;
    for (char* t = strtok_r(sp, " \t\r\n", &s2); t; t = strtok_r(NULL, " \t\r\n", &s2))
        snprintf(m->names[m->ng + m->ns++], NL, "%s", t);
    free(work);
    for (int i = 0; i < m->ns; ++i) { m->sigma[m->ng + i] = 1.0; m->th0[i] = 0.0; }
    work = strdup(txt);
    char site_attr[256];
    char* site = tag_body(work, "SITE", NULL, site_attr, sizeof site_attr);
    if (site) {
        char* sw = strdup(site);
        char* co = tag_body(sw, "COORDINATION", NULL, NULL, 0);
        if (co) {
            char* s3 = NULL;
            for (char* t = strtok_r(co, ",", &s3); t; t = strtok_r(NULL, ",", &s3)) {
                char* eq = strchr(t, '='); if (!eq) continue; *eq = 0;
                int k = find_species(m, trim(t), m->ng, m->ng + m->ns);
                if (k >= 0) m->sigma[k] = atof(eq + 1);
            }
        }
        free(sw); sw = strdup(site);
        char* de = tag_body(sw, "DENSITY", NULL, NULL, 0);
        if (de) m->site_density = atof(trim(de));
        free(sw); sw = strdup(site);
        char* in = tag_body(sw, "INITIAL", NULL, NULL, 0);
        if (in) {
            char* s3 = NULL;
            for (char* t = strtok_r(in, ",", &s3); t; t = strtok_r(NULL, ",", &s3)) {
                char* eq = strchr(t, '='); if (!eq) continue; *eq = 0;
                int k = find_species(m, trim(t), m->ng, m->ng + m->ns);
                if (k >= 0) m->th0[k - m->ng] = atof(eq + 1);
            }
        }
        free(sw);
    }
    free(work);
    /* reactions */
    int cap = 64; m->sr = (srxn_t*)calloc((size_t)cap, sizeof(srxn_t)); m->nrs = 0;
    int ids[512]; /* reaction id -> index */
    for (int i = 0; i < 512; ++i) ids[i] = -1;
    for (int pass = 0; pass < 2; ++pass) {
        work = strdup(txt);
        char* blk = tag_body(work, pass == 0 ? "STICK" : "ARRHENIUS", NULL, NULL, 0);
        char* p = blk;
        while (p) {
            char attrs[128];
            char* after = NULL;
            char* body = tag_body(p, "RXN", &after, attrs, sizeof attrs);
            if (!body) break;
            int id = -1; char* ip = strstr(attrs, "ID=\"");
            if (ip) id = atoi(ip + 4);
            char* at = strchr(body, '@');
            if (!at) { seterr("surface rxn without '@'"); return -1; }
            *at = 0;
            if (m->nrs == cap) { cap *= 2; m->sr = (srxn_t*)realloc(m->sr, (size_t)cap * sizeof(srxn_t)); }
            srxn_t* r = &m->sr[m->nrs]; memset(r, 0, sizeof *r);
            char* arrow = strstr(body, "=>");
            if (!arrow) { seterr("surface rxn without '=>'"); return -1; }
            *arrow = 0;
            if (parse_surf_side(m, body, r->f, &r->nf) || parse_surf_side(m, arrow + 2, r->p, &r->np)) return -1;
            double a = 0, b = 0, e = 0;
            int nv = sscanf(at + 1, "%lf %lf %lf", &a, &b, &e);
            if (pass == 0) {
                r->stick = 1; r->A = a; r->stick_gas = -1;
                for (int i = 0; i < r->nf; ++i) if (r->f[i] < m->ng) r->stick_gas = r->f[i];
                if (r->stick_gas < 0) { seterr("sticking rxn without gas species"); return -1; }
            } else {
                if (nv < 3) { seterr("arrhenius rxn needs A b E"); return -1; }
                int ms = 0, mg = 0;
                for (int i = 0; i < r->nf; ++i) { if (r->f[i] >= m->ng) ms++; else mg++; }
                r->A = a * pow(1e-4, ms - 1) * pow(1e-6, mg);
                r->b = b; r->Ea = e * efac;
            }
            if (id >= 0 && id < 512) ids[id] = m->nrs;
            m->nrs++;
            p = after;
        }
        free(work);
    }
    /* coverage dependencies: <coverage id="12 20 21">co(ni)=-50</coverage> */
    work = strdup(txt);
    char* p = work;
    for (;;) {
        char attrs[128]; char* after = NULL;
        char* body = tag_body(p, "COVERAGE", &after, attrs, sizeof attrs);
        if (!body) break;
        char* eq = strchr(body, '=');
        if (eq) {
            *eq = 0;
            int k = find_species(m, trim(body), m->ng, m->ng + m->ns);
            double eps = atof(eq + 1) * efac;
            char* ip = strstr(attrs, "ID=\"");
            if (ip && k >= 0) {
                char idl[128]; snprintf(idl, sizeof idl, "%s", ip + 4);
                char* q = strchr(idl, '"'); if (q) *q = 0;
                char* s3 = NULL;
                for (char* t = strtok_r(idl, " ", &s3); t; t = strtok_r(NULL, " ", &s3)) {
                    int id = atoi(t);
                    if (id >= 0 && id < 512 && ids[id] >= 0) {
                        srxn_t* r = &m->sr[ids[id]];
                        r->cov_sp[r->ncov] = k; r->cov_eps[r->ncov++] = eps;
                    }
                }
            }
        }
        p = after;
    }
    free(work);
    free(txt);
    return 0;
}

orc_mech* orc_load(const char* gas_mech, const char* therm, const char* surf_mech,
                   const char* gas_species, int conv, double p_std) {
    orc_mech* m = (orc_mech*)calloc(1, sizeof(orc_mech));
    m->conv = conv; m->p_std = p_std > 0 ? p_std : 1e5;
    if (gas_mech) {
        if (load_chemkin(m, gas_mech)) { orc_free(m); return NULL; }
    } else if (gas_species) {
        char* w = strdup(gas_species); char* s2 = NULL;
        for (char* t = strtok_r(w, " \t\n", &s2); t; t = strtok_r(NULL, " \t\n", &s2)) {
            snprintf(m->names[m->ng], NL, "%s", t); upcase(m->names[m->ng]); m->ng++;
        }
        free(w);
    }
    thermo_t* tab = NULL;
    int nt = load_thermo(therm, &tab);
    if (nt < 0 || attach_thermo(m, tab, nt)) { free(tab); orc_free(m); return NULL; }
    free(tab);
    if (surf_mech && load_surface(m, surf_mech)) { orc_free(m); return NULL; }
    return m;
}

void orc_free(orc_mech* m) {
    if (!m) return;
    for (int r = 0; r < m->nrg; ++r) free(m->gr[r].eff);
    free(m->gr); free(m->sr); free(m);
}

/* ----------------------------------------------------------------------------------- */
/* temperature-only quantities (T is constant per reactor: ConstantParams, :14-17)      */
/* ----------------------------------------------------------------------------------- */
typedef struct {
    double T;
    double *kf, *kr, *k0, *fc;   /* [nrg] */
    double *ks;                  /* [nrs] arrhenius k without coverage term; sticking factor */
} tcache_t;

static double g_over_RT(const thermo_t* t, double T) {
    const double* a = (T < t->tmid) ? t->lo : t->hi;
    double lT = log(T);
    double h = a[0] + a[1] * T / 2 + a[2] * T * T / 3 + a[3] * T * T * T / 4 + a[4] * T * T * T * T / 5 + a[5] / T;
    double s = a[0] * lT + a[1] * T + a[2] * T * T / 2 + a[3] * T * T * T / 3 + a[4] * T * T * T * T / 4 + a[6];
    return h - s;
}

static void tcache_init(const orc_mech* m, double T, tcache_t* c) {
    c->T = T;
    c->kf = (double*)malloc(sizeof(double) * (size_t)(4 * m->nrg + m->nrs + 1));
    c->kr = c->kf + m->nrg; c->k0 = c->kr + m->nrg; c->fc = c->k0 + m->nrg; c->ks = c->fc + m->nrg;
    double g[MAXSP];
    for (int k = 0; k < m->ng; ++k) g[k] = g_over_RT(&m->th[k], T);
    double lT = log(T);
    for (int i = 0; i < m->nrg; ++i) {
        const grxn_t* r = &m->gr[i];
        c->kf[i] = r->A * exp(r->b * lT - r->EoR / T);
        c->kr[i] = 0.0;
        if (r->rev) {
            double dg = 0;
            for (int e = 0; e < r->nr; ++e) dg += g[r->r[e]];
            for (int e = 0; e < r->nf; ++e) dg -= g[r->f[e]];
            double Kc = exp(-dg) * pow(m->p_std / (R_GAS * T), r->dnu);
            /* GasphaseReactions evaluates rates in mol/cm3 but Kc = Kp (p0/RT)^dnu in mol/m3 */
            if (m->conv & ORC_CONV_KC_UNIT_SLIP) Kc *= pow(1e6, r->dnu);
            c->kr[i] = c->kf[i] / Kc;
        }
        c->k0[i] = 0; c->fc[i] = 1;
        if (r->tb == 2) {
            c->k0[i] = r->A0 * exp(r->b0 * lT - r->E0oR / T);
            if (r->troe) {
                double fc = (1 - r->ta) * exp(-T / r->t3) + r->ta * exp(-T / r->t1);
                if (r->has_t2) fc += exp(-r->t2 / T);
                c->fc[i] = fc;
            }
        }
    }
    for (int i = 0; i < m->nrs; ++i) {
        const srxn_t* r = &m->sr[i];
        if (r->stick) c->ks[i] = r->A * sqrt(R_GAS * T / (2 * M_PI * m->M[r->stick_gas]));
        else c->ks[i] = r->A * pow(T, r->b) * exp(-r->Ea / (R_GAS * T));
    }
}
static void tcache_free(tcache_t* c) { free(c->kf); }

/* falloff factor fac = Pr/(1+Pr)*F and d(fac)/d[M] */
static void falloff(const orc_mech* m, const grxn_t* r, const tcache_t* c, int i, double Mc, double* fac, double* dfac) {
    double kinf = c->kf[i], k0 = c->k0[i];
    double Pr = k0 * Mc / kinf;
    double F = 1.0, g = 0.0;
    if (r->troe) {
        double Prs = Pr > 1e-300 ? Pr : 1e-300;
        double lfc = log10(c->fc[i]);
        double L = log10(Prs);
        double cc = ((m->conv & ORC_CONV_TROE_C4) ? -4.0 : -0.4) - 0.67 * lfc, nn = 0.75 - 1.27 * lfc;
        double den = nn - 0.14 * (L + cc);
        double f1 = (L + cc) / den;
        double lF = lfc / (1 + f1 * f1);
        F = pow(10.0, lF);
        double df1 = nn / (den * den);
        g = -lfc * 2 * f1 / ((1 + f1 * f1) * (1 + f1 * f1)) * df1; /* d log10F / d log10Pr */
    }
    *fac = Pr / (1 + Pr) * F;
    /* d fac/dPr = F/(1+Pr)^2 + F*g/(1+Pr); dPr/d[M] = k0/kinf */
    *dfac = (F / ((1 + Pr) * (1 + Pr)) + F * g / (1 + Pr)) * (k0 / kinf);
}

/* diagnostic hook (scripts/parity_outliers.py, diag_spread.py): every rate of progress -- for a gas
 * reaction each direction kf Pf, kr Pb separately -- times (1 +- eps), the sign from a hash of (call,
 * reaction, direction): the few-ulp differences of an RHS implementation that evaluates the same
 * formulas in another order, amplified by CVODE's DQ Jacobian (inc ~ 1e-8 |y|). 0 = off. */
static double g_rop_jitter = 0.0;
/* per thread, and touched only while the jitter is on: a shared counter written by every OpenMP thread on
 * every RHS call was a data race and put all threads on one cache line (16-thread baseline -80 %, r04) */
static _Thread_local unsigned long long g_rop_calls = 0;
/* deterministic streams: each integration restarts the counter at (seed, reactor index) << 24, so a
 * reactor's jitter sequence does not depend on the thread that ran it or on what that thread ran
 * before (orc_integrate_batch passes the batch index; single integrations use index 0) */
static unsigned long long g_rop_seed = 0;
static _Thread_local unsigned long long g_rop_reactor = 0;
void orc_set_rop_jitter(double eps) { g_rop_jitter = eps; }
void orc_set_rop_jitter_seed(unsigned long long seed) { g_rop_seed = seed; }
static inline double rop_jit(int i) {   /* sign from a splitmix64 finaliser of (call, reaction): every bit mixed */
    unsigned long long h = g_rop_calls * 0x9E3779B97F4A7C15ull + (unsigned long long)(i + 1) * 0xC2B2AE3D27D4EB4Full;
    h = (h ^ (h >> 30)) * 0xBF58476D1CE4E5B9ull;
    h = (h ^ (h >> 27)) * 0x94D049BB133111EBull;
    h ^= h >> 31;
    return (h & 1) ? g_rop_jitter : -g_rop_jitter;
}

/* gas rates of progress q[nrg] from concentrations c[ng] */
static void gas_rop(const orc_mech* m, const tcache_t* tc, const double* c, double* q) {
    for (int i = 0; i < m->nrg; ++i) {
        const grxn_t* r = &m->gr[i];
        double Pf = 1, Pb = 1;
        for (int e = 0; e < r->nf; ++e) Pf *= c[r->f[e]];
        for (int e = 0; e < r->nr; ++e) Pb *= c[r->r[e]];
        /* jitter (diag): each direction's rate separately, so a net rate near partial equilibrium
         * (kf Pf ~ kr Pb) carries the absolute rounding of its terms, as a reordered RHS would */
        double D = g_rop_jitter != 0.0
                       ? r->fmul * tc->kf[i] * Pf * (1.0 + rop_jit(2 * i)) - r->rmul * tc->kr[i] * Pb * (1.0 + rop_jit(2 * i + 1))
                       : r->fmul * tc->kf[i] * Pf - r->rmul * tc->kr[i] * Pb;
        if (r->tb) {
            double Mc = 0;
            for (int k = 0; k < m->ng; ++k) Mc += r->eff[k] * c[k];
            if (r->tb == 1) D *= Mc;
            else {
                double fac, dfac; falloff(m, r, tc, i, Mc, &fac, &dfac);
                D *= fac;
                if (m->conv & ORC_CONV_FALLOFF_XM) D *= Mc * 1e-6;   /* [M] in mol/cm3 */
            }
        }
        q[i] = D;
    }
    if (g_rop_jitter != 0.0) g_rop_calls++;
}

static void surf_rop(const orc_mech* m, const tcache_t* tc, const double* c, const double* th, double* q) {
    double G = m->site_density * 1e4; /* mol/m2 */
    double RT = R_GAS * tc->T;
    for (int i = 0; i < m->nrs; ++i) {
        const srxn_t* r = &m->sr[i];
        double k = tc->ks[i];
        if (r->ncov) {
            double s = 0;
            for (int j = 0; j < r->ncov; ++j) s += r->cov_eps[j] * th[r->cov_sp[j] - m->ng];
            k *= exp(-s / RT);
        }
        double P = 1;
        for (int e = 0; e < r->nf; ++e) {
            int s = r->f[e];
            if (s < m->ng) P *= c[s];
            else P *= r->stick ? th[s - m->ng] : th[s - m->ng] * G / m->sigma[s];
        }
        q[i] = g_rop_jitter != 0.0 ? k * P * (1.0 + rop_jit(100000 + i)) : k * P;
    }
    if (g_rop_jitter != 0.0) g_rop_calls++;
}

static void conc_from_x(const orc_mech* m, double T, double p, const double* x, double* c) {
    for (int k = 0; k < m->ng; ++k) c[k] = p * x[k] / (R_GAS * T);
}

void orc_rop(const orc_mech* m, double T, double p, const double* x, const double* th, double* qg, double* qs) {
    tcache_t tc; tcache_init(m, T, &tc);
    double c[MAXSP]; conc_from_x(m, T, p, x, c);
    if (qg && m->nrg) gas_rop(m, &tc, c, qg);
    if (qs && m->nrs) surf_rop(m, &tc, c, th, qs);
    tcache_free(&tc);
}

static void rates_tc(const orc_mech* m, const tcache_t* tc, double p, const double* x, const double* th,
                     double* wdot, double* sdot) {
    double c[MAXSP]; conc_from_x(m, tc->T, p, x, c);
    int n = m->ng + m->ns;
    double q[1024];
    if (wdot) {
        for (int k = 0; k < m->ng; ++k) wdot[k] = 0;
        if (m->nrg) {
            gas_rop(m, tc, c, q);
            for (int i = 0; i < m->nrg; ++i) {
                const grxn_t* r = &m->gr[i];
                for (int e = 0; e < r->nf; ++e) wdot[r->f[e]] -= q[i];
                for (int e = 0; e < r->nr; ++e) wdot[r->r[e]] += q[i];
            }
        }
    }
    if (sdot) {
        for (int k = 0; k < n; ++k) sdot[k] = 0;
        if (m->nrs) {
            surf_rop(m, tc, c, th, q);
            for (int i = 0; i < m->nrs; ++i) {
                const srxn_t* r = &m->sr[i];
                for (int e = 0; e < r->nf; ++e) sdot[r->f[e]] -= q[i];
                for (int e = 0; e < r->np; ++e) sdot[r->p[e]] += q[i];
            }
        }
    }
}

void orc_rates(const orc_mech* m, double T, double p, const double* x, const double* th, double* wdot, double* sdot) {
    tcache_t tc; tcache_init(m, T, &tc);
    rates_tc(m, &tc, p, x, th, wdot, sdot);
    tcache_free(&tc);
}

void orc_initial_state(const orc_mech* m, double T, double p, const double* x, double* u) {
    /* IdealGas.density: rho = p*Mbar/(R T); molefrac_to_massfrac: Y = x M / Mbar */
    double Mb = 0;
    for (int k = 0; k < m->ng; ++k) Mb += x[k] * m->M[k];
    double rho = p * Mb / (R_GAS * T);
    for (int k = 0; k < m->ng; ++k) u[k] = (x[k] * m->M[k] / Mb) * rho;
    for (int i = 0; i < m->ns; ++i) u[m->ng + i] = m->th0[i];
}

/* residual! (src/BatchReactor.jl:312-376) */
static void rhs_tc(const orc_mech* m, const tcache_t* tc, double Asv, const double* u, double* du,
                   double* p_out, double* x_out) {
    int ng = m->ng, ns = m->ns;
    double rho = 0;
    for (int k = 0; k < ng; ++k) rho += u[k];                       /* :326 */
    double Y[MAXSP], x[MAXSP], s = 0;
    for (int k = 0; k < ng; ++k) { Y[k] = u[k] / rho; s += Y[k] / m->M[k]; }  /* :328 */
    for (int k = 0; k < ng; ++k) x[k] = (Y[k] / m->M[k]) / s;       /* massfrac_to_molefrac! */
    double Mb = 0;
    for (int k = 0; k < ng; ++k) Mb += x[k] * m->M[k];              /* average_molwt */
    double p = rho * R_GAS * tc->T / Mb;                            /* :338 / :353 */
    double sdot[MAXSP], wdot[MAXSP];
    for (int k = 0; k < ng + ns; ++k) sdot[k] = 0;
    for (int k = 0; k < ng; ++k) wdot[k] = 0;
    if (ns) {
        rates_tc(m, tc, p, x, u + ng, NULL, sdot);                  /* :344 */
        for (int k = 0; k < ng + ns; ++k) sdot[k] *= Asv;           /* :345 (whole vector) */
    }
    if (m->nrg) rates_tc(m, tc, p, x, NULL, wdot, NULL);            /* :355 */
    for (int k = 0; k < ng; ++k) du[k] = (sdot[k] + wdot[k]) * m->M[k];   /* :363-370 */
    double Gcm = m->site_density;
    for (int i = 0; i < ns; ++i) {
        double sd = sdot[ng + i];
        if (m->conv & ORC_CONV_DOC_COVG) sd /= Asv;
        du[ng + i] = sd * m->sigma[ng + i] / (Gcm * 1e4);          /* :367 / :370 */
    }
    if (p_out) *p_out = p;
    if (x_out) for (int k = 0; k < ng; ++k) x_out[k] = x[k];
}

void orc_rhs(const orc_mech* m, double T, double Asv, const double* u, double* du, double* p_out, double* x_out) {
    tcache_t tc; tcache_init(m, T, &tc);
    rhs_tc(m, &tc, Asv, u, du, p_out, x_out);
    tcache_free(&tc);
}

/* analytic Jacobian d(du)/du, row-major (new work: the reference uses CVODE's DQ Jacobian) */
static void jac_tc(const orc_mech* m, const tcache_t* tc, double Asv, const double* u, double* J) {
    int ng = m->ng, ns = m->ns, n = ng + ns;
    for (int i = 0; i < n * n; ++i) J[i] = 0;
    double c[MAXSP];
    for (int k = 0; k < ng; ++k) c[k] = u[k] / m->M[k];   /* = p x_k/(RT) algebraically */
    const double* th = u + ng;
    double dq[MAXSP];
    int touched[MAXSP], nt;
    for (int i = 0; i < m->nrg; ++i) {
        const grxn_t* r = &m->gr[i];
        for (int k = 0; k < ng; ++k) dq[k] = 0;
        double Pf = 1, Pb = 1;
        for (int e = 0; e < r->nf; ++e) Pf *= c[r->f[e]];
        for (int e = 0; e < r->nr; ++e) Pb *= c[r->r[e]];
        double kf = r->fmul * tc->kf[i], kr = r->rmul * tc->kr[i];
        double D = kf * Pf - kr * Pb;
        double pre = 1, coefM = 0, Mc = 0;
        if (r->tb) {
            for (int k = 0; k < ng; ++k) Mc += r->eff[k] * c[k];
            if (r->tb == 1) { pre = Mc; coefM = 1; }
            else {
                double fac, dfac; falloff(m, r, tc, i, Mc, &fac, &dfac);
                int xm = (m->conv & ORC_CONV_FALLOFF_XM) != 0;
                const double xs = 1e-6;
                pre = fac * (xm ? Mc * xs : 1.0);
                coefM = dfac * (xm ? Mc * xs : 1.0) + (xm ? fac * xs : 0.0);
            }
        }
        for (int e = 0; e < r->nf; ++e) {
            double pr = kf;
            for (int e2 = 0; e2 < r->nf; ++e2) if (e2 != e) pr *= c[r->f[e2]];
            dq[r->f[e]] += pre * pr;
        }
        for (int e = 0; e < r->nr; ++e) {
            double pr = kr;
            for (int e2 = 0; e2 < r->nr; ++e2) if (e2 != e) pr *= c[r->r[e2]];
            dq[r->r[e]] -= pre * pr;
        }
        if (r->tb) for (int k = 0; k < ng; ++k) dq[k] += D * coefM * r->eff[k];
        /* rows touched */
        nt = 0;
        double nu[MAXSP];
        for (int e = 0; e < r->nf; ++e) { int s = r->f[e]; int f = 0; for (int t = 0; t < nt; ++t) if (touched[t] == s) f = 1; if (!f) { touched[nt++] = s; nu[s] = 0; } nu[s] -= 1; }
        for (int e = 0; e < r->nr; ++e) { int s = r->r[e]; int f = 0; for (int t = 0; t < nt; ++t) if (touched[t] == s) f = 1; if (!f) { touched[nt++] = s; nu[s] = 0; } nu[s] += 1; }
        for (int t = 0; t < nt; ++t) {
            int k = touched[t];
            if (nu[k] == 0) continue;
            for (int j = 0; j < ng; ++j) J[k * n + j] += m->M[k] * nu[k] * dq[j] / m->M[j];
        }
    }
    if (m->nrs) {
        double G = m->site_density * 1e4, RT = R_GAS * tc->T;
        double asv_th = (m->conv & ORC_CONV_DOC_COVG) ? 1.0 : Asv;
        for (int i = 0; i < m->nrs; ++i) {
            const srxn_t* r = &m->sr[i];
            double k = tc->ks[i];
            if (r->ncov) {
                double s = 0;
                for (int j = 0; j < r->ncov; ++j) s += r->cov_eps[j] * th[r->cov_sp[j] - ng];
                k *= exp(-s / RT);
            }
            double conc[MAXE], dconc[MAXE];
            for (int e = 0; e < r->nf; ++e) {
                int s = r->f[e];
                if (s < ng) { conc[e] = c[s]; dconc[e] = 1.0 / m->M[s]; }
                else if (r->stick) { conc[e] = th[s - ng]; dconc[e] = 1.0; }
                else { conc[e] = th[s - ng] * G / m->sigma[s]; dconc[e] = G / m->sigma[s]; }
            }
            double P = 1; for (int e = 0; e < r->nf; ++e) P *= conc[e];
            double q = k * P;
            double dqv[MAXSP]; for (int j = 0; j < n; ++j) dqv[j] = 0;
            for (int e = 0; e < r->nf; ++e) {
                double pr = k;
                for (int e2 = 0; e2 < r->nf; ++e2) if (e2 != e) pr *= conc[e2];
                dqv[r->f[e]] += pr * dconc[e];
            }
            for (int j = 0; j < r->ncov; ++j) dqv[r->cov_sp[j]] += q * (-r->cov_eps[j] / RT);
            for (int e = 0; e < r->nf + r->np; ++e) {
                int s = e < r->nf ? r->f[e] : r->p[e - r->nf];
                double nu = e < r->nf ? -1.0 : 1.0;
                double rowf = s < ng ? m->M[s] * Asv : asv_th * m->sigma[s] / G;
                for (int j = 0; j < n; ++j) J[s * n + j] += rowf * nu * dqv[j];
            }
        }
    }
}

void orc_jac(const orc_mech* m, double T, double Asv, const double* u, double* J) {
    tcache_t tc; tcache_init(m, T, &tc);
    jac_tc(m, &tc, Asv, u, J);
    tcache_free(&tc);
}

/* ----------------------------------------------------------------------------------- */
/* CVODE 5.x restatement (cvode.c / cvode_ls.c / sunnonlinsol_newton.c / sundials_dense) */
/* ----------------------------------------------------------------------------------- */
#define QMAX 5
#define L_MAX (QMAX + 1)
#define HLB_FACTOR 100.0
#define HUB_FACTOR 0.1
#define H_BIAS 0.5
#define MAX_ITERS 4
#define ETAMX1 10000.0
#define ETAMX2 10.0
#define ETAMX3 10.0
#define ETAMXF 0.2
#define ETAMIN 0.1
#define ETACF 0.25
#define ADDON 1e-6
#define BIAS1 6.0
#define BIAS2 6.0
#define BIAS3 10.0
#define ONEPSM 1.000001
#define SMALL_NST 10
#define MXNCF 10
#define MXNEF 7
#define MXNEF1 3
#define SMALL_NEF 2
#define LONG_WAIT 10
#define NLS_MAXCOR 3
#define CRDOWN 0.3
#define DGMAX 0.3
#define RDIV 2.0
#define MSBP 20
#define CORTES 0.1
#define THRESH 1.5
#define FUZZ_FACTOR 100.0
#define LS_MSBJ 51
#define LS_DGMAX 0.2
#define MIN_INC_MULT 1000.0

enum { FIRST_CALL, PREV_CONV_FAIL, PREV_ERR_FAIL };
enum { NO_FAILURES, FAIL_BAD_J, FAIL_OTHER };

typedef struct {
    const orc_mech* m; const tcache_t* tc; double Asv;
    int n; double rtol, atol; int analytic;
    double* zn[L_MAX + 1];
    double *ewt, *y, *acor, *tempv, *ftemp, *delta;
    double *savedJ, *A; int* piv;
    double tn, h, hprime, hscale, eta, etamax, hmin, hmax_inv, hu;
    double tau[L_MAX + 1], tq[6], l[L_MAX];
    double rl1, gamma, gammap, gamrat, crate, delp, acnrm, saved_tq5;
    double etaq, etaqm1, etaqp1;
    int q, qprime, L, qwait, indx_acor;
    long nst, nfe, nsetups, nje, nni, ncfn, netf, nstlp, nstlj, nscon, nfeDQ;
    double uround;
    int jcur;
    int convfail;
    /* last-RHS state for save_data semantics */
    double p_last, x_last[MAXSP], th_last[MAXSP];
    double tstop;
    int lu_map[MAXSP];      /* step -> original row of the previous factorization (diagnostic) */
    int lu_nmap;
} cv_t;

static double wrms(const cv_t* cv, const double* x) {
    double s = 0;
    for (int i = 0; i < cv->n; ++i) { double t = x[i] * cv->ewt[i]; s += t * t; }
    return sqrt(s / cv->n);
}
static void fcall(cv_t* cv, const double* y, double* f) {
    rhs_tc(cv->m, cv->tc, cv->Asv, y, f, &cv->p_last, cv->x_last);
    for (int i = 0; i < cv->m->ns; ++i) cv->th_last[i] = y[cv->m->ng + i];
}
static void set_ewt(cv_t* cv, const double* y) {
    for (int i = 0; i < cv->n; ++i) cv->ewt[i] = 1.0 / (cv->rtol * fabs(y[i]) + cv->atol);
}

/* SUNDIALS denseGETRF / denseGETRS on column-major a[j*n+i] */
static int getrf(double* a, int n, int* p) {
    for (int k = 0; k < n; ++k) {
        double* ck = a + (size_t)k * n;
        int l = k;
        for (int i = k + 1; i < n; ++i) if (fabs(ck[i]) > fabs(ck[l])) l = i;
        p[k] = l;
        if (ck[l] == 0.0) return k + 1;
        if (l != k) for (int i = 0; i < n; ++i) { double t = a[(size_t)i * n + l]; a[(size_t)i * n + l] = a[(size_t)i * n + k]; a[(size_t)i * n + k] = t; }
        double mult = 1.0 / ck[k];
        for (int i = k + 1; i < n; ++i) ck[i] *= mult;
        for (int j = k + 1; j < n; ++j) {
            double* cj = a + (size_t)j * n;
            double akj = cj[k];
            if (akj != 0.0) for (int i = k + 1; i < n; ++i) cj[i] -= akj * ck[i];
        }
    }
    return 0;
}
static void getrs(const double* a, int n, const int* p, double* b) {
    for (int k = 0; k < n; ++k) { int pk = p[k]; if (pk != k) { double t = b[k]; b[k] = b[pk]; b[pk] = t; } }
    for (int k = 0; k < n - 1; ++k) { const double* ck = a + (size_t)k * n; double bk = b[k]; for (int i = k + 1; i < n; ++i) b[i] -= ck[i] * bk; }
    for (int k = n - 1; k > 0; --k) { const double* ck = a + (size_t)k * n; b[k] /= ck[k]; double bk = b[k]; for (int i = 0; i < k; ++i) b[i] -= ck[i] * bk; }
    b[0] /= a[0];
}

static void dq_jac(cv_t* cv, const double* y, const double* fy, double* Jc /* col-major */) {
    int n = cv->n;
    double srur = sqrt(cv->uround);
    double fnorm = wrms(cv, fy);
    double minInc = (fnorm != 0.0) ? (MIN_INC_MULT * fabs(cv->h) * cv->uround * n * fnorm) : 1.0;
    double* yy = cv->tempv; /* scratch copy */
    for (int i = 0; i < n; ++i) yy[i] = y[i];
    double* ft = (double*)malloc(sizeof(double) * (size_t)n);
    /* test hook (scripts/diag_spread.py): a relative perturbation of the DQ increments, the size of
       the rounding differences between two implementations of cvLsDenseDQJac */
    static double jitter = -1.0;
    if (jitter < 0.0) { const char* e = getenv("ORC_DQ_JITTER"); jitter = e ? atof(e) : 0.0; }
    for (int j = 0; j < n; ++j) {
        double ys = yy[j];
        double inc = fmax(srur * fabs(ys), minInc / cv->ewt[j]) * (1.0 + ((j & 1) ? jitter : -jitter));
        yy[j] += inc;
        fcall(cv, yy, ft);
        cv->nfeDQ++;
        yy[j] = ys;
        double ii = 1.0 / inc;
        for (int i = 0; i < n; ++i) Jc[(size_t)j * n + i] = ii * ft[i] - ii * fy[i];
    }
    free(ft);
}

/* diagnostic (scripts/lu_order_stats.py; off unless orc_lu_diag(1)): how often a factorization's
 * pivot sequence differs from the previous factorization's of the same integration, i.e. how often
 * an engine that loads the rows in the previous pivot order meets a pivot off its step's position,
 * and how many such steps (row interchanges needed, denseGETRF on the reordered rows) */
static _Thread_local int g_lu_diag = 0;
static _Thread_local long g_lu_stat[8];   /* factorizations, deviating ones, steps, interchanges,
                                              sum of interchange steps k, sum of k - (k >= 32 ? 32 : 0),
                                              first factorization's interchanges, steps whose column max
                                              shares its high word with another candidate */
void orc_lu_diag(int on) { g_lu_diag = on; for (int i = 0; i < 8; ++i) g_lu_stat[i] = 0; }
void orc_lu_stats(long* out8) { for (int i = 0; i < 8; ++i) out8[i] = g_lu_stat[i]; }
static void lu_order_diag(cv_t* cv) {
    int n = cv->n;
    double* B = (double*)malloc(sizeof(double) * (size_t)n * n);
    int* pv = (int*)malloc(sizeof(int) * (size_t)n);
    int map[MAXSP];
    if (cv->lu_nmap != n) { for (int i = 0; i < n; ++i) cv->lu_map[i] = i; cv->lu_nmap = n; }
    /* rows in the previous pivot order: position s holds original row lu_map[s] */
    for (int j = 0; j < n; ++j) for (int s = 0; s < n; ++s) B[(size_t)j * n + s] = cv->A[(size_t)j * n + cv->lu_map[s]];
    for (int s = 0; s < n; ++s) map[s] = cv->lu_map[s];
    int sw = 0;
    {   /* hi-word ties of the column max among the candidates, in the reordered matrix (a copy) */
        double* Cc = (double*)malloc(sizeof(double) * (size_t)n * n);
        int* pc = (int*)malloc(sizeof(int) * (size_t)n);
        memcpy(Cc, B, sizeof(double) * (size_t)n * n);
        for (int k = 0; k < n; ++k) {
            double* ck = Cc + (size_t)k * n;
            int l = k;
            for (int i = k + 1; i < n; ++i) if (fabs(ck[i]) > fabs(ck[l])) l = i;
            unsigned long long bl; double al = fabs(ck[l]); memcpy(&bl, &al, 8);
            int cnt = 0;
            for (int i = k; i < n; ++i) { double ai = fabs(ck[i]); unsigned long long bi; memcpy(&bi, &ai, 8); if ((bi >> 32) == (bl >> 32)) ++cnt; }
            if (cnt > 1) g_lu_stat[7]++;
            if (ck[l] == 0.0) break;
            if (l != k) for (int i = 0; i < n; ++i) { double t = Cc[(size_t)i * n + l]; Cc[(size_t)i * n + l] = Cc[(size_t)i * n + k]; Cc[(size_t)i * n + k] = t; }
            double mult = 1.0 / ck[k];
            for (int i = k + 1; i < n; ++i) ck[i] *= mult;
            for (int j = k + 1; j < n; ++j) { double* cj = Cc + (size_t)j * n; double akj = cj[k]; if (akj != 0.0) for (int i = k + 1; i < n; ++i) cj[i] -= akj * ck[i]; }
        }
        free(Cc); free(pc);
    }
    if (getrf(B, n, pv) == 0) {
        for (int k = 0; k < n; ++k) if (pv[k] != k) {
            int t = map[k]; map[k] = map[pv[k]]; map[pv[k]] = t; ++sw;
            g_lu_stat[4] += k; g_lu_stat[5] += k >= 32 ? k - 32 : k;
        }
    }
    if (g_lu_stat[0] == 0) g_lu_stat[6] = sw;
    g_lu_stat[0]++; g_lu_stat[1] += sw > 0; g_lu_stat[2] += n; g_lu_stat[3] += sw;
    for (int s = 0; s < n; ++s) cv->lu_map[s] = map[s];
    free(B); free(pv);
}

/* cvLsSetup: build A = I - gamma*J (maybe reusing savedJ) and factor */
static int ls_setup(cv_t* cv, int convfail, const double* ypred, const double* fpred) {
    int n = cv->n;
    double dgamma = fabs(cv->gamma / cv->gammap - 1.0);
    int jbad = (cv->nst == 0) || (cv->nst > cv->nstlj + LS_MSBJ) ||
               ((convfail == FAIL_BAD_J) && (dgamma < LS_DGMAX)) || (convfail == FAIL_OTHER);
    if (!jbad) {
        cv->jcur = 0;
        memcpy(cv->A, cv->savedJ, sizeof(double) * (size_t)n * n);
    } else {
        cv->jcur = 1; cv->nje++; cv->nstlj = cv->nst;
        if (cv->analytic) {
            double* Jr = (double*)malloc(sizeof(double) * (size_t)n * n);
            jac_tc(cv->m, cv->tc, cv->Asv, ypred, Jr);
            for (int i = 0; i < n; ++i) for (int j = 0; j < n; ++j) cv->A[(size_t)j * n + i] = Jr[(size_t)i * n + j];
            free(Jr);
        } else {
            dq_jac(cv, ypred, fpred, cv->A);
        }
        memcpy(cv->savedJ, cv->A, sizeof(double) * (size_t)n * n);
    }
    for (size_t i = 0; i < (size_t)n * n; ++i) cv->A[i] *= -cv->gamma;
    for (int i = 0; i < n; ++i) cv->A[(size_t)i * n + i] += 1.0;
    if (g_lu_diag) lu_order_diag(cv);
    return getrf(cv->A, n, cv->piv);
}

static void cv_rescale(cv_t* cv) {
    double factor = cv->eta;
    for (int j = 1; j <= cv->q; ++j) { for (int i = 0; i < cv->n; ++i) cv->zn[j][i] *= factor; factor *= cv->eta; }
    cv->h = cv->hscale * cv->eta; cv->hscale = cv->h; cv->nscon = 0;
}
static void cv_predict(cv_t* cv) {
    cv->tn += cv->h;
    if ((cv->tn - cv->tstop) * cv->h > 0) cv->tn = cv->tstop;
    for (int k = 1; k <= cv->q; ++k)
        for (int j = cv->q; j >= k; --j)
            for (int i = 0; i < cv->n; ++i) cv->zn[j - 1][i] += cv->zn[j][i];
}
static void cv_restore(cv_t* cv, double saved_t) {
    cv->tn = saved_t;
    for (int k = 1; k <= cv->q; ++k)
        for (int j = cv->q; j >= k; --j)
            for (int i = 0; i < cv->n; ++i) cv->zn[j - 1][i] -= cv->zn[j][i];
}
static void set_tq_bdf(cv_t* cv, double hsum, double alpha0, double alpha0_hat, double xi_inv, double xistar_inv) {
    int q = cv->q;
    double A1 = 1.0 - alpha0_hat + alpha0;
    double A2 = 1.0 + q * A1;
    cv->tq[2] = fabs(A1 / (alpha0 * A2));
    cv->tq[5] = fabs(A2 * xistar_inv / (cv->l[q] * xi_inv));
    if (cv->qwait == 1) {
        if (q > 1) {
            double C = xistar_inv / cv->l[q];
            double A3 = alpha0 + 1.0 / q;
            double A4 = alpha0_hat + xi_inv;
            double Cpinv = (1.0 - A4 + A3) / A3;
            cv->tq[1] = fabs(C * Cpinv);
        } else cv->tq[1] = 1.0;
        hsum += cv->tau[q];
        xi_inv = cv->h / hsum;
        double A5 = alpha0 - (1.0 / (q + 1));
        double A6 = alpha0_hat - xi_inv;
        double Cppinv = (1.0 - A6 + A5) / A2;
        cv->tq[3] = fabs(Cppinv / (xi_inv * (q + 2) * A5));
    }
    cv->tq[4] = CORTES / cv->tq[2];
}
static void cv_set(cv_t* cv) {
    int q = cv->q;
    double* l = cv->l;
    double xi_inv = 1.0, xistar_inv = 1.0;
    l[0] = l[1] = 1.0;
    for (int i = 2; i <= q; ++i) l[i] = 0.0;
    double alpha0 = -1.0, alpha0_hat = -1.0, hsum = cv->h;
    if (q > 1) {
        for (int j = 2; j < q; ++j) {
            hsum += cv->tau[j - 1];
            xi_inv = cv->h / hsum;
            alpha0 -= 1.0 / j;
            for (int i = j; i >= 1; --i) l[i] += l[i - 1] * xi_inv;
        }
        alpha0 -= 1.0 / q;
        xistar_inv = -l[1] - alpha0;
        hsum += cv->tau[q - 1];
        xi_inv = cv->h / hsum;
        alpha0_hat = -l[1] - xi_inv;
        for (int i = q; i >= 1; --i) l[i] += l[i - 1] * xistar_inv;
    }
    set_tq_bdf(cv, hsum, alpha0, alpha0_hat, xi_inv, xistar_inv);
    cv->rl1 = 1.0 / l[1];
    cv->gamma = cv->h * cv->rl1;
    if (cv->nst == 0) cv->gammap = cv->gamma;
    cv->gamrat = (cv->nst > 0) ? cv->gamma / cv->gammap : 1.0;
}
static void increase_bdf(cv_t* cv) {
    double* l = cv->l; int q = cv->q;
    for (int i = 0; i <= QMAX; ++i) l[i] = 0.0;
    l[2] = 1.0;
    double alpha1 = 1.0, prod = 1.0, xiold = 1.0, alpha0 = -1.0, hsum = cv->hscale;
    if (q > 1) {
        for (int j = 1; j < q; ++j) {
            hsum += cv->tau[j + 1];
            double xi = hsum / cv->hscale;
            prod *= xi;
            alpha0 -= 1.0 / (j + 1);
            alpha1 += 1.0 / xi;
            for (int i = j + 2; i >= 2; --i) l[i] = l[i] * xiold + l[i - 1];
            xiold = xi;
        }
    }
    double A1 = (-alpha0 - alpha1) / prod;
    int L = q + 1;
    for (int i = 0; i < cv->n; ++i) cv->zn[L][i] = A1 * cv->zn[cv->indx_acor][i];
    for (int j = 2; j <= q; ++j) for (int i = 0; i < cv->n; ++i) cv->zn[j][i] += l[j] * cv->zn[L][i];
}
static void decrease_bdf(cv_t* cv) {
    double* l = cv->l; int q = cv->q;
    for (int i = 0; i <= QMAX; ++i) l[i] = 0.0;
    l[2] = 1.0;
    double hsum = 0.0;
    for (int j = 1; j <= q - 2; ++j) {
        hsum += cv->tau[j];
        double xi = hsum / cv->hscale;
        for (int i = j + 2; i >= 2; --i) l[i] = l[i] * xi + l[i - 1];
    }
    for (int j = 2; j < q; ++j) for (int i = 0; i < cv->n; ++i) cv->zn[j][i] -= l[j] * cv->zn[q][i];
}
static void adjust_order(cv_t* cv, int dq) {
    if ((cv->q == 2) && (dq != 1)) return;   /* cvAdjustOrder guard */
    if (dq == 1) increase_bdf(cv); else decrease_bdf(cv);
}

/* SUNNonlinSol_Newton + cvNls; returns 0 ok, >0 recoverable conv failure, <0 unrecoverable */
static int cv_nls(cv_t* cv, int nflag) {
    int n = cv->n;
    int convfail = ((nflag == FIRST_CALL) || (nflag == PREV_ERR_FAIL)) ? NO_FAILURES : FAIL_OTHER;
    int callSetup = (nflag == PREV_CONV_FAIL) || (nflag == PREV_ERR_FAIL) || (cv->nst == 0) ||
                    (cv->nst >= cv->nstlp + MSBP) || (fabs(cv->gamrat - 1.0) > DGMAX);
    double* ycor = cv->acor;
    for (int i = 0; i < n; ++i) ycor[i] = 0.0;
    double tol = cv->tq[4];
    int jbad = 0, jcur = 0, ret = 0;
    for (;;) {
        /* residual */
        for (int i = 0; i < n; ++i) cv->y[i] = cv->zn[0][i] + ycor[i];
        fcall(cv, cv->y, cv->ftemp); cv->nfe++;
        for (int i = 0; i < n; ++i) cv->delta[i] = (cv->rl1 * cv->zn[1][i] + ycor[i]) - cv->gamma * cv->ftemp[i];
        if (callSetup) {
            int cf = jbad ? FAIL_BAD_J : convfail;
            int lr = ls_setup(cv, cf, cv->y, cv->ftemp);
            cv->nsetups++;
            jcur = cv->jcur;
            cv->gamrat = 1.0; cv->gammap = cv->gamma; cv->crate = 1.0; cv->nstlp = cv->nst;
            if (lr) { ret = 1; /* recoverable LU failure: singular */ goto fail_ls; }
        }
        int m = 0;
        for (;;) {
            cv->nni++;
            for (int i = 0; i < n; ++i) cv->delta[i] = -cv->delta[i];
            getrs(cv->A, n, cv->piv, cv->delta);
            if (cv->gamrat != 1.0) { double s = 2.0 / (1.0 + cv->gamrat); for (int i = 0; i < n; ++i) cv->delta[i] *= s; }
            for (int i = 0; i < n; ++i) ycor[i] += cv->delta[i];
            /* cvNlsConvTest */
            double del = wrms(cv, cv->delta);
            if (m > 0) cv->crate = fmax(CRDOWN * cv->crate, del / cv->delp);
            double dcon = del * fmin(1.0, cv->crate) / tol;
            if (dcon <= 1.0) {
                cv->acnrm = (m == 0) ? del : wrms(cv, ycor);
                for (int i = 0; i < n; ++i) cv->y[i] = cv->zn[0][i] + ycor[i];
                cv->jcur = 0;
                return 0;
            }
            if ((m >= 1) && (del > RDIV * cv->delp)) { ret = 1; break; }
            cv->delp = del;
            m++;
            if (m >= NLS_MAXCOR) { ret = 1; break; }
            for (int i = 0; i < n; ++i) cv->y[i] = cv->zn[0][i] + ycor[i];
            fcall(cv, cv->y, cv->ftemp); cv->nfe++;
            for (int i = 0; i < n; ++i) cv->delta[i] = (cv->rl1 * cv->zn[1][i] + ycor[i]) - cv->gamma * cv->ftemp[i];
        }
        if (ret > 0 && !jcur) {
            callSetup = 1; jbad = 1;
            for (int i = 0; i < n; ++i) ycor[i] = 0.0;
            continue;
        }
        break;
    }
    for (int i = 0; i < n; ++i) cv->y[i] = cv->zn[0][i] + ycor[i];
    return ret;
fail_ls:
    return 2; /* lsetup failure (singular matrix) treated as recoverable conv failure */
}

static void complete_step(cv_t* cv) {
    cv->nst++; cv->nscon++;
    cv->hu = cv->h;
    for (int i = cv->q; i >= 2; --i) cv->tau[i] = cv->tau[i - 1];
    if ((cv->q == 1) && (cv->nst > 1)) cv->tau[2] = cv->tau[1];
    cv->tau[1] = cv->h;
    for (int j = 0; j <= cv->q; ++j) for (int i = 0; i < cv->n; ++i) cv->zn[j][i] += cv->l[j] * cv->acor[i];
    cv->qwait--;
    if ((cv->qwait == 1) && (cv->q != QMAX)) {
        memcpy(cv->zn[QMAX], cv->acor, sizeof(double) * (size_t)cv->n);
        cv->saved_tq5 = cv->tq[5];
        cv->indx_acor = QMAX;
    }
}
static void set_eta(cv_t* cv) {
    if (cv->eta < THRESH) { cv->eta = 1.0; cv->hprime = cv->h; }
    else {
        cv->eta = fmin(cv->eta, cv->etamax);
        cv->eta /= fmax(1.0, fabs(cv->h) * cv->hmax_inv * cv->eta);
        cv->hprime = cv->h * cv->eta;
        if (cv->qprime < cv->q) cv->nscon = 0;
    }
}
static void prepare_next_step(cv_t* cv, double dsm) {
    if (cv->etamax == 1.0) {
        cv->qwait = cv->qwait > 2 ? cv->qwait : 2;
        cv->qprime = cv->q; cv->hprime = cv->h; cv->eta = 1.0;
        return;
    }
    cv->etaq = 1.0 / (pow(BIAS2 * dsm, 1.0 / cv->L) + ADDON);
    if (cv->qwait != 0) { cv->eta = cv->etaq; cv->qprime = cv->q; set_eta(cv); return; }
    cv->qwait = 2;
    cv->etaqm1 = 0.0;
    if (cv->q > 1) {
        double ddn = wrms(cv, cv->zn[cv->q]) * cv->tq[1];
        cv->etaqm1 = 1.0 / (pow(BIAS1 * ddn, 1.0 / cv->q) + ADDON);
    }
    cv->etaqp1 = 0.0;
    if (cv->q != QMAX && cv->saved_tq5 != 0.0) {
        double cquot = (cv->tq[5] / cv->saved_tq5) * pow(cv->h / cv->tau[2], (double)cv->L);
        for (int i = 0; i < cv->n; ++i) cv->tempv[i] = cv->acor[i] - cquot * cv->zn[QMAX][i];
        double dup = wrms(cv, cv->tempv) * cv->tq[3];
        cv->etaqp1 = 1.0 / (pow(BIAS3 * dup, 1.0 / (cv->L + 1)) + ADDON);
    }
    /* cvChooseEta */
    double etam = fmax(cv->etaqm1, fmax(cv->etaq, cv->etaqp1));
    if (etam < THRESH) { cv->eta = 1.0; cv->qprime = cv->q; }
    else if (etam == cv->etaq) { cv->eta = cv->etaq; cv->qprime = cv->q; }
    else if (etam == cv->etaqm1) { cv->eta = cv->etaqm1; cv->qprime = cv->q - 1; }
    else {
        cv->eta = cv->etaqp1; cv->qprime = cv->q + 1;
        memcpy(cv->zn[QMAX], cv->acor, sizeof(double) * (size_t)cv->n);
    }
    set_eta(cv);
}

/* one cvStep; returns 0 ok, <0 failure */
static int cv_step(cv_t* cv) {
    double saved_t = cv->tn;
    int ncf = 0, nef = 0, nflag = FIRST_CALL;
    double dsm = 0;
    if ((cv->nst > 0) && (cv->hprime != cv->h)) {
        if (cv->qprime != cv->q) {
            adjust_order(cv, cv->qprime - cv->q);
            cv->q = cv->qprime; cv->L = cv->q + 1; cv->qwait = cv->L;
        }
        cv_rescale(cv);
    }
    for (;;) {
        cv_predict(cv);
        cv_set(cv);
        int r = cv_nls(cv, nflag);
        if (r != 0) {
            /* cvHandleNFlag */
            cv->ncfn++;
            cv_restore(cv, saved_t);
            ncf++;
            cv->etamax = 1.0;
            if ((fabs(cv->h) <= cv->hmin * ONEPSM) || (ncf == MXNCF)) return -4;
            cv->eta = fmax(ETACF, cv->hmin / fabs(cv->h));
            nflag = PREV_CONV_FAIL;
            cv_rescale(cv);
            continue;
        }
        /* cvDoErrorTest */
        dsm = cv->acnrm * cv->tq[2];
        if (dsm <= 1.0) break;
        nef++; cv->netf++; nflag = PREV_ERR_FAIL;
        cv_restore(cv, saved_t);
        if ((fabs(cv->h) <= cv->hmin * ONEPSM) || (nef == MXNEF)) return -3;
        cv->etamax = 1.0;
        if (nef <= MXNEF1) {
            cv->eta = 1.0 / (pow(BIAS2 * dsm, 1.0 / cv->L) + ADDON);
            cv->eta = fmax(ETAMIN, fmax(cv->eta, cv->hmin / fabs(cv->h)));
            if (nef >= SMALL_NEF) cv->eta = fmin(cv->eta, ETAMXF);
            cv_rescale(cv);
            continue;
        }
        if (cv->q > 1) {
            cv->eta = fmax(ETAMIN, cv->hmin / fabs(cv->h));
            adjust_order(cv, -1);
            cv->L = cv->q; cv->q--; cv->qwait = cv->L;
            cv_rescale(cv);
            continue;
        }
        cv->eta = fmax(ETAMIN, cv->hmin / fabs(cv->h));
        cv->h *= cv->eta; cv->hscale = cv->h; cv->qwait = LONG_WAIT; cv->nscon = 0;
        fcall(cv, cv->zn[0], cv->tempv); cv->nfe++;
        for (int i = 0; i < cv->n; ++i) cv->zn[1][i] = cv->h * cv->tempv[i];
    }
    complete_step(cv);
    prepare_next_step(cv, dsm);
    cv->etamax = (cv->nst <= SMALL_NST) ? ETAMX2 : ETAMX3;
    for (int i = 0; i < cv->n; ++i) cv->acor[i] *= cv->tq[2];
    return 0;
}

/* cvHin */
static void cv_hin(cv_t* cv, double tout) {
    int n = cv->n;
    double t0 = cv->tn;
    double tdist = fabs(tout - t0);
    double tround = cv->uround * fmax(fabs(t0), fabs(tout));
    double hlb = HLB_FACTOR * tround;
    /* cvUpperBoundH0 */
    double hub_inv = 0;
    for (int i = 0; i < n; ++i) {
        double t1 = HUB_FACTOR * fabs(cv->zn[0][i]) + 1.0 / cv->ewt[i];
        double r = fabs(cv->zn[1][i]) / t1;
        if (r > hub_inv) hub_inv = r;
    }
    double hub = HUB_FACTOR * tdist;
    if (hub * hub_inv > 1.0) hub = 1.0 / hub_inv;
    double hg = sqrt(hlb * hub);
    if (hub < hlb) { cv->h = hg; return; }
    int hnewOK = 0;
    double hnew = hg, yddnrm = 0;
    for (int count1 = 1; count1 <= MAX_ITERS; ++count1) {
        /* cvYddNorm */
        for (int i = 0; i < n; ++i) cv->y[i] = hg * cv->zn[1][i] + cv->zn[0][i];
        fcall(cv, cv->y, cv->tempv); cv->nfe++;
        for (int i = 0; i < n; ++i) cv->tempv[i] = (cv->tempv[i] - cv->zn[1][i]) * (1.0 / hg);
        yddnrm = wrms(cv, cv->tempv);
        if (hnewOK || count1 == MAX_ITERS) { hnew = hg; break; }
        hnew = (yddnrm * hub * hub > 2.0) ? sqrt(2.0 / yddnrm) : sqrt(hg * hub);
        double hrat = hnew / hg;
        if ((hrat > 0.5) && (hrat < 2.0)) hnewOK = 1;
        if ((count1 > 1) && (hrat > 2.0)) { hnew = hg; hnewOK = 1; }
        hg = hnew;
    }
    double h0 = H_BIAS * hnew;
    if (h0 < hlb) h0 = hlb;
    if (h0 > hub) h0 = hub;
    cv->h = h0;
}

/* CVodeGetDky, k = 0 */
static void get_dky(const cv_t* cv, double t, double* y) {
    double s = (t - cv->tn) / cv->h;
    for (int i = 0; i < cv->n; ++i) y[i] = cv->zn[cv->q][i];
    for (int j = cv->q - 1; j >= 0; --j) for (int i = 0; i < cv->n; ++i) y[i] = cv->zn[j][i] + s * y[i];
}

static int integrate_impl(const orc_mech* m, double T, double Asv, double* u, double tf,
                          const orc_opts* o, orc_stats* st, orc_step_cb cb, void* user,
                          int nout, const double* tout, double* yout);

int orc_integrate(const orc_mech* m, double T, double Asv, double* u, double tf,
                  const orc_opts* o, orc_stats* st, orc_step_cb cb, void* user) {
    return integrate_impl(m, T, Asv, u, tf, o, st, cb, user, 0, NULL, NULL);
}

/* CVode(..., CV_NORMAL) at each output time: the solver steps past tout and interpolates with
 * CVodeGetDky(tout, 0) (Nordsieck polynomial); the step sequence is the same as without outputs. */
int orc_integrate_out(const orc_mech* m, double T, double Asv, double* u, double tf, const orc_opts* o,
                      orc_stats* st, int nout, const double* tout, double* yout) {
    return integrate_impl(m, T, Asv, u, tf, o, st, NULL, NULL, nout, tout, yout);
}

static int integrate_impl(const orc_mech* m, double T, double Asv, double* u, double tf,
                          const orc_opts* o, orc_stats* st, orc_step_cb cb, void* user,
                          int nout, const double* tout, double* yout) {
    tcache_t tc; tcache_init(m, T, &tc);
    g_rop_calls = ((g_rop_seed << 20) + g_rop_reactor) << 24;
    cv_t cvs; cv_t* cv = &cvs; memset(cv, 0, sizeof *cv);
    int n = m->ng + m->ns;
    cv->m = m; cv->tc = &tc; cv->Asv = Asv; cv->n = n;
    cv->rtol = o ? o->rtol : 1e-6; cv->atol = o ? o->atol : 1e-10;
    cv->analytic = o ? o->analytic_jac : 0;
    long mxstep = (o && o->max_steps > 0) ? o->max_steps : 100000;
    cv->hmax_inv = (o && o->hmax > 0) ? 1.0 / o->hmax : 0.0;
    cv->uround = DBL_EPSILON;
    double* mem = (double*)calloc((size_t)(L_MAX + 1 + 7) * n + 2 * (size_t)n * n, sizeof(double));
    for (int j = 0; j <= L_MAX; ++j) cv->zn[j] = mem + (size_t)j * n;
    double* p = mem + (size_t)(L_MAX + 1) * n;
    cv->ewt = p; p += n; cv->y = p; p += n; cv->acor = p; p += n; cv->tempv = p; p += n;
    cv->ftemp = p; p += n; cv->delta = p; p += n; p += n;
    cv->savedJ = p; p += (size_t)n * n; cv->A = p;
    cv->piv = (int*)calloc((size_t)n, sizeof(int));
    /* CVodeInit */
    cv->tn = 0.0; cv->tstop = tf;
    memcpy(cv->zn[0], u, sizeof(double) * (size_t)n);
    cv->q = 1; cv->L = 2; cv->qwait = cv->L; cv->etamax = ETAMX1; cv->crate = 1.0;
    cv->indx_acor = QMAX;
    /* initial callback: save_data at t0 sees the untouched state (p_initial, x0) */
    if (cb) {
        double rho = 0, x[MAXSP], s = 0;
        for (int k = 0; k < m->ng; ++k) rho += u[k];
        for (int k = 0; k < m->ng; ++k) s += (u[k] / rho) / m->M[k];
        for (int k = 0; k < m->ng; ++k) x[k] = ((u[k] / rho) / m->M[k]) / s;
        double Mb = 0; for (int k = 0; k < m->ng; ++k) Mb += x[k] * m->M[k];
        cb(user, 0.0, u, rho * R_GAS * T / Mb, x, u + m->ng);
    }
    /* cvInitialSetup + first-call part of CVode */
    set_ewt(cv, cv->zn[0]);
    fcall(cv, cv->zn[0], cv->zn[1]); cv->nfe++;
    cv_hin(cv, tf);
    if (cv->hmax_inv > 0) { double rh = fabs(cv->h) * cv->hmax_inv; if (rh > 1.0) cv->h /= rh; }
    if ((cv->tn + cv->h - cv->tstop) * cv->h > 0.0) cv->h = (cv->tstop - cv->tn) * (1.0 - 4.0 * cv->uround);
    cv->hscale = cv->h; cv->hprime = cv->h;
    for (int i = 0; i < n; ++i) cv->zn[1][i] *= cv->h;
    double ufac = o ? o->unstable_factor : 0.0, uscale = 0.0;   /* <= 0: NaN check only */
    for (int i = 0; i < n; ++i) uscale += fabs(u[i]);
    int status = 0;
    long nstloc = 0;
    int iout = 0;
    int ign = (o && o->ignition_species > 0 && o->ignition_species <= m->ng) ? o->ignition_species - 1 : -1;
    double ign_x = 0.0, ign_t = 0.0, ign_rate = -INFINITY, t_ign = NAN, ign_dt = NAN;
    if (ign >= 0) { double g = 0; for (int k = 0; k < m->ng; ++k) g += u[k] / m->M[k]; ign_x = (u[ign] / m->M[ign]) / g; }
    while (iout < nout && tout[iout] <= 0.0) { memcpy(yout + (size_t)iout * n, u, sizeof(double) * (size_t)n); ++iout; }
    for (;;) {
        if (cv->nst > 0) set_ewt(cv, cv->zn[0]);
        if (nstloc >= mxstep) { status = -1; break; }
        int kf = cv_step(cv);
        if (kf) { status = kf; break; }
        nstloc++;
        {   /* SciML unstable_check (NaN), or the opt-in runaway test */
            double mx = 0.0;
            for (int i = 0; i < n; ++i) { double a = fabs(cv->zn[0][i]); mx = fmax(mx, a == a ? a : INFINITY); }
            if (!(mx < INFINITY) || (ufac > 0.0 && mx > ufac * uscale)) { status = -7; break; }
        }
        if (ign >= 0) {   /* ignition marker on the accepted states */
            double g = 0; for (int k = 0; k < m->ng; ++k) g += cv->zn[0][k] / m->M[k];
            double x = (cv->zn[0][ign] / m->M[ign]) / g, r = (x - ign_x) / (cv->tn - ign_t);
            if (r > ign_rate) { ign_rate = r; t_ign = 0.5 * (ign_t + cv->tn); ign_dt = cv->tn - ign_t; }
            ign_x = x; ign_t = cv->tn;
        }
        while (iout < nout && tout[iout] <= cv->tn) { get_dky(cv, tout[iout], yout + (size_t)iout * n); ++iout; }
        double troundoff = FUZZ_FACTOR * cv->uround * (fabs(cv->tn) + fabs(cv->h));
        if (fabs(cv->tn - cv->tstop) <= troundoff) {
            while (iout < nout && tout[iout] <= cv->tstop) { get_dky(cv, tout[iout], yout + (size_t)iout * n); ++iout; }
            get_dky(cv, cv->tstop, u);
            if (cb) cb(user, cv->tstop, u, cv->p_last, cv->x_last, cv->th_last);
            break;
        }
        if ((cv->tn + cv->hprime - cv->tstop) * cv->h > 0.0) {
            cv->hprime = (cv->tstop - cv->tn) * (1.0 - 4.0 * cv->uround);
            cv->eta = cv->hprime / cv->h;
        }
        if (cb) cb(user, cv->tn, cv->zn[0], cv->p_last, cv->x_last, cv->th_last);
    }
    if (status) memcpy(u, cv->zn[0], sizeof(double) * (size_t)n);
    if (st) {
        st->nsteps = cv->nst; st->nfe = cv->nfe; st->nje = cv->nje; st->nsetups = cv->nsetups;
        st->nni = cv->nni; st->ncfn = cv->ncfn; st->netf = cv->netf; st->nfeDQ = cv->nfeDQ;
        st->status = status; st->qlast = cv->q; st->hlast = cv->h; st->tcur = cv->tn;
        st->t_ign = ign >= 0 ? t_ign : NAN; st->ign_rate = ign >= 0 ? ign_rate : NAN;
        st->ign_dt = ign >= 0 ? ign_dt : NAN;
    }
    free(cv->piv); free(mem); tcache_free(&tc);
    return status;
}

int orc_integrate_batch(const orc_mech* m, int N, const double* T, const double* Asv, double* u,
                        const double* tf, const orc_opts* o, orc_stats* st, int nthreads) {
    return orc_integrate_batch_out(m, N, T, Asv, u, tf, o, st, nthreads, 0, NULL, NULL);
}

int orc_integrate_batch_out(const orc_mech* m, int N, const double* T, const double* Asv, double* u,
                            const double* tf, const orc_opts* o, orc_stats* st, int nthreads,
                            int nout, const double* tout, double* yout) {
    int n = m->ng + m->ns;
    int bad = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : bad)
#endif
    for (int i = 0; i < N; ++i) {
        g_rop_reactor = (unsigned long long)i;
        int r = integrate_impl(m, T[i], Asv ? Asv[i] : 1.0, u + (size_t)i * n, tf[i], o, st ? &st[i] : NULL, NULL, NULL,
                               nout, tout, yout ? yout + (size_t)i * nout * n : NULL);
        g_rop_reactor = 0;
        if (r) bad++;
    }
    (void)nthreads;
    return bad;
}
