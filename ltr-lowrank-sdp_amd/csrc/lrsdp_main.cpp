// lrsdp_main.cpp -- drop-in replacement for the LoRADS CLI binary
// (`LoRADS_v_2_0_1-alpha <file.dat-s> --flag value ... --jsonfile out.json`) that
// benchmark.py (benchmark.py:240-262) and dataset/run_lorads.sh call.  Same
// argv contract as src_semi/main.c:256-348 (argv[1] = instance, getopt_long
// flags main.c:125-154, unknown flags ignored, exit code 0), plus the three
// flags the reference never implemented (--rankSchedule, --nearStallFactor,
// --disableOracle) and --device.  The solve runs on the MI355X
// through liblrsdp.so (include/lrsdp.h).
#include <getopt.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lrsdp.h"

extern "C" int lrs_set_log_path(lrs_ctx *ctx, const char *path);

static bool parse_schedule(const char *path, std::vector<int> &out) {
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    std::string s;
    char buf[4096];
    size_t n;
    while ((n = fread(buf, 1, sizeof(buf), f)) > 0) s.append(buf, n);
    fclose(f);
    size_t k = s.find("\"rank_schedule\"");
    if (k == std::string::npos) return false;
    k = s.find('[', k);
    size_t e = s.find(']', k);
    if (k == std::string::npos || e == std::string::npos) return false;
    const char *p = s.c_str() + k + 1, *end = s.c_str() + e;
    while (p < end) {
        char *q;
        long v = strtol(p, &q, 10);
        if (q == p) { p++; continue; }
        out.push_back((int)v);
        p = q;
    }
    return !out.empty();
}

static std::string problem_name(const char *path) {   // set_problem_name, lorads_logging.c
    std::string s(path);
    size_t sl = s.find_last_of('/');
    if (sl != std::string::npos) s = s.substr(sl + 1);
    size_t dot = s.find('.');
    if (dot != std::string::npos) s = s.substr(0, dot);
    return s;
}

int main(int argc, char **argv) {
    lrs_params p;
    lrs_params_default(&p);
    p.verbose = 1;
    const char *logFile = nullptr, *jsonFile = nullptr, *schedFile = nullptr;
    int device = 0;
    static struct option opts[] = {
        {"logfile", required_argument, 0, 1025}, {"jsonfile", required_argument, 0, 1026},
        {"initRho", required_argument, 0, 1000}, {"rhoMax", required_argument, 0, 1001},
        {"rhoCellingALM", required_argument, 0, 1002}, {"rhoCellingADMM", required_argument, 0, 1003},
        {"maxALMIter", required_argument, 0, 1004}, {"maxADMMIter", required_argument, 0, 1005},
        {"timesLogRank", required_argument, 0, 1006}, {"fixedRank", required_argument, 0, 1022},
        {"initRank", required_argument, 0, 1023}, {"rhoFreq", required_argument, 0, 1007},
        {"rhoFactor", required_argument, 0, 1008}, {"ALMRhoFactor", required_argument, 0, 1009},
        {"rankUpdateFactor", required_argument, 0, 1024}, {"phase1Tol", required_argument, 0, 1010},
        {"phase2Tol", required_argument, 0, 1011}, {"timeSecLimit", required_argument, 0, 1012},
        {"heuristicFactor", required_argument, 0, 1013}, {"lbfgsListLength", required_argument, 0, 1014},
        {"endTauTol", required_argument, 0, 1015}, {"endALMSubTol", required_argument, 0, 1016},
        {"l2Rescaling", required_argument, 0, 1017}, {"reoptLevel", required_argument, 0, 1018},
        {"dyrankLevel", required_argument, 0, 1019}, {"highAccMode", required_argument, 0, 1020},
        {"oracleRankNaive", no_argument, 0, 1021},
        {"rankSchedule", required_argument, 0, 2000}, {"nearStallFactor", required_argument, 0, 2001},
        {"disableOracle", no_argument, 0, 2002}, {"device", required_argument, 0, 2003},
        {"quiet", no_argument, 0, 2004}, {0, 0, 0, 0}};
    if (argc < 2) {
        fprintf(stderr, "usage: %s <file.dat-s> [--flag value ...]\n", argv[0]);
        return 0;
    }
    const char *fname = argv[1];
    int opt, li = 0;
    while ((opt = getopt_long(argc, argv, "r:", opts, &li)) != -1) {
        switch (opt) {
        case 1025: logFile = optarg; break;
        case 1026: jsonFile = optarg; break;
        case 1000: p.initRho = atof(optarg); break;
        case 1001: p.rhoMax = atof(optarg); break;
        case 1002: p.rhoCellingALM = atof(optarg); break;
        case 1003: p.rhoCellingADMM = atof(optarg); break;
        case 1004: p.maxALMIter = atoi(optarg); break;
        case 1005: p.maxADMMIter = atoi(optarg); break;
        case 1006: p.timesLogRank = atof(optarg); break;
        case 1022: p.fixedRank = atoi(optarg); break;
        case 1023: p.initRank = atoi(optarg); break;
        case 1007: p.rhoFreq = atoi(optarg); break;
        case 1008: p.rhoFactor = atof(optarg); break;
        case 1009: p.ALMRhoFactor = atof(optarg); break;
        case 1024: p.rankUpdateFactor = atof(optarg); break;
        case 1010: p.phase1Tol = atof(optarg); break;
        case 1011: p.phase2Tol = atof(optarg); break;
        case 1012: p.timeSecLimit = atof(optarg); break;
        case 1013: p.heuristicFactor = atof(optarg); break;
        case 1014: p.lbfgsListLength = atoi(optarg); break;
        case 1015: p.endTauTol = atof(optarg); break;
        case 1016: p.endALMSubTol = atof(optarg); break;
        case 1017: p.l2Rescaling = atoi(optarg); break;
        case 1018: p.reoptLevel = atoi(optarg); break;
        case 1019: p.dyrankLevel = atoi(optarg); break;
        case 1020: p.highAccMode = atoi(optarg); break;
        case 1021: p.oracleRankNaive = 1; break;
        case 2000: schedFile = optarg; break;
        case 2001: p.nearStallFactor = atof(optarg); break;
        case 2002: p.disableOracle = 1; break;
        case 2003: device = atoi(optarg); break;
        case 2004: p.verbose = 0; break;
        default: break;   // unknown flags: getopt already printed a message; ignored like main.c
        }
    }
    std::vector<int> sched;
    if (schedFile) {
        if (parse_schedule(schedFile, sched)) {
            p.rankSchedule = sched.data();
            p.rankScheduleLen = (int)sched.size();
        } else {
            fprintf(stderr, "[lrsdp] could not parse rank schedule %s; ignored\n", schedFile);
        }
    }
    if (p.lbfgsListLength < 1) {   // the reference's ring needs one node at least (data/lorads_solver.c:686-706)
        fprintf(stderr, "[lrsdp] lbfgsListLength %d < 1; using 2\n", p.lbfgsListLength);
        p.lbfgsListLength = 2;
    }
    printf("-----------------------------------------------------------\n");
    printf("  LoRADS-compatible low-rank SDP solver on MI355X (%s)\n", lrs_version());
    printf("-----------------------------------------------------------\n");
    lrs_ctx *ctx = nullptr;
    if (lrs_ctx_create(device, &ctx)) {
        fprintf(stderr, "[lrsdp] %s\n", lrs_last_error());
        return 0;
    }
    if (logFile) lrs_set_log_path(ctx, logFile);
    double tread = 0;
    if (lrs_load_sdpa(ctx, fname, &tread)) {
        fprintf(stderr, "[lrsdp] %s\n", lrs_last_error());
        lrs_ctx_destroy(ctx);
        return 0;   // main.c:383-385 exits 0 on read failure too
    }
    int m = 0, K = 0;
    lrs_problem_info(ctx, &m, &K, nullptr, nullptr, nullptr);
    printf("Reading SDPA file in %f seconds \n", tread);
    printf("nConstrs = %d, sdp nBlks = %d, lp Cols = %d\n", m, K, 0);
    lrs_result r;
    if (lrs_solve(ctx, &p, &r)) {
        fprintf(stderr, "[lrsdp] solve failed: %s\n", lrs_last_error());
        lrs_ctx_destroy(ctx);
        return 0;
    }
    printf("-----------------------------------------------------------------------\n");
    // LORADSEndProgram, data/lorads_solver.c:1307-1333
    if (r.status == 3) printf("End Program due to reaching `the maximum number of iterations`:\n");
    else if (r.status == 1) printf("End Program due to reaching `Official terminate criteria`:\n");
    else if (r.status == 2) printf("End Program due to reaching `final terminate criteria`:\n");
    else if (r.status == 4) printf("End Program since time limit.\n");
    else printf("End Program but the status is unknown, please notify the authors\n");
    const double dinf = r.dinf < 0 ? 0.0 : r.dinf, dinf_inf = r.dinf_inf < 0 ? 0.0 : r.dinf_inf;
    printf("Objective function Value are:\n");
    printf("\t 1.Primal Objective:            : %10.6e\n", r.pobj);
    printf("\t 2.Dual Objective:              : %10.6e\n", r.dobj);
    printf("Dimacs Error are:\n");
    printf("\t 1.Constraint Violation(1)      : %10.6e\n", r.pinf);
    printf("\t 2.Dual Infeasibility(1)        : %10.6e\n", dinf);
    printf("\t 3.Primal Dual Gap              : %10.6e\n", r.gap);
    printf("\t 4.Primal Variable Semidefinite : %10.6e\n", 0.0);
    printf("\t 5.Constraint Violation(Inf)    : %10.6e\n", r.pinf_inf);
    printf("\t 6.Dual Infeasibility(Inf)      : %10.6e\n", dinf_inf);
    printf("-----------------------------------------------------------------------\n");
    printf("ALM inner iterations: %ld, ALM time: %f s, ADMM iterations: %ld\n", r.alm_inner, r.alm_time, r.admm_iter);
    printf("all_time: %f\n", r.solve_time);
    if (jsonFile) {
        std::string pid = problem_name(fname);
        if (lrs_write_json(ctx, jsonFile, pid.c_str(), fname, &r, &p))
            fprintf(stderr, "[lrsdp] %s\n", lrs_last_error());
        else
            printf("JSON output written to: %s\n", jsonFile);
    }
    lrs_ctx_destroy(ctx);
    return 0;
}
