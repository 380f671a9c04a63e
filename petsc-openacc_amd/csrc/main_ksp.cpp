// main_ksp.cpp — the reference's KSP driver (/root/reference/src/main_ksp.cpp)
// restated over the C ABI: build the 3-D Poisson system of helper.cpp, solve
// it with device-resident CG, print the same result block
// (main_ksp.cpp:124-129), so scripts/generate_plots.py's regex still parses it.
//
//   main_ksp [-config FILE] [-da_grid_x N] [-da_grid_y N] [-da_grid_z N]
//            [-ksp_rtol R] [-ksp_atol A] [-ksp_max_it K] [-pc_type jacobi|none|gamg]
//            [-ksp_norm_type preconditioned|unpreconditioned|natural]
//            [-pc_gamg_threshold T] [-pc_gamg_agg_nsmooths S]
//            [-pc_gamg_coarse_eq_limit C] [-pc_mg_levels L] [-pc_gamg_square_graph G]
//            [-aijhip_gamg_coarsen 1|0] [-aijhip_gamg_eig_ksp 1|0] [-aijhip_host_assembly]
//
// Options come from the command line and from a PETSc options file
// (`-key value` per line, '#' comments; PetscOptionsInsertFile,
// main_ksp.cpp:74-77); command-line values win. Grid defaults 100^3
// (main_ksp.cpp:33-35 "-100" = 100, overridable).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "aijhip.h"
#include "aijhip_harness.h"
#include "aijhip_ksp.h"

namespace {

double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void parse_file(const std::string &path, std::map<std::string, std::string> &opt) {
    std::ifstream f(path);
    if (!f) {
        std::fprintf(stderr, "main_ksp: cannot open options file %s\n", path.c_str());
        std::exit(1);
    }
    std::string line;
    while (std::getline(f, line)) {
        const auto h = line.find('#');
        if (h != std::string::npos) line.resize(h);
        std::istringstream is(line);
        std::string key, val;
        if (!(is >> key) || key[0] != '-') continue;
        is >> val;
        if (!opt.count(key)) opt[key] = val;
    }
}

#define CHK(call)                                                                       \
    do {                                                                                \
        int rc_ = (call);                                                               \
        if (rc_) {                                                                      \
            std::fprintf(stderr, "main_ksp: %s failed (%d): %s\n", #call, rc_,          \
                         aijhip_last_error());                                          \
            std::exit(rc_);                                                             \
        }                                                                               \
    } while (0)

#define HCHK(call)                                                                      \
    do {                                                                                \
        hipError_t e_ = (call);                                                         \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "main_ksp: %s: %s\n", #call, hipGetErrorString(e_));   \
            std::exit(3);                                                               \
        }                                                                               \
    } while (0)

}  // namespace

int main(int argc, char **argv) {
    std::map<std::string, std::string> opt;
    std::string config;
    for (int i = 1; i < argc; ++i) {
        std::string k = argv[i];
        if (k.size() < 2 || k[0] != '-') continue;
        std::string v = (i + 1 < argc && argv[i + 1][0] != '-') ? argv[++i] : "";
        if (k == "-config") config = v;
        else opt[k] = v;
    }
    if (!config.empty()) parse_file(config, opt);
    auto geti = [&](const char *k, long d) { return opt.count(k) ? std::atol(opt[k].c_str()) : d; };
    auto getd = [&](const char *k, double d) { return opt.count(k) ? std::atof(opt[k].c_str()) : d; };
    auto gets = [&](const char *k, const char *d) { return opt.count(k) ? opt[k] : std::string(d); };

    const int32_t nx = (int32_t)geti("-da_grid_x", 100), ny = (int32_t)geti("-da_grid_y", 100),
                  nz = (int32_t)geti("-da_grid_z", 100);
    const std::string ksp_type = gets("-ksp_type", "cg");
    if (ksp_type != "cg") {
        std::fprintf(stderr, "main_ksp: -ksp_type %s not supported (cg only)\n", ksp_type.c_str());
        return 1;
    }
    std::string pc_type = gets("-pc_type", "jacobi");
    if (pc_type == "bjacobi") pc_type = "jacobi";  // one block per rank + jacobi sub-PC
    int pc = pc_type == "none" ? AIJHIP_PC_NONE : pc_type == "gamg" ? AIJHIP_PC_GAMG : AIJHIP_PC_JACOBI;
    if (pc_type != "none" && pc_type != "jacobi" && pc_type != "gamg") {
        std::fprintf(stderr, "main_ksp: -pc_type %s not supported\n", pc_type.c_str());
        return 1;
    }
    aijhip_gamg_params_t gp;
    aijhip_gamg_params_default(&gp);
    if (pc == AIJHIP_PC_GAMG) {
        // PETSc_SolverOptions_GAMG.info:6-21. The level smoother and coarse
        // solver are fixed to that file's choice (Richardson(1) + Jacobi,
        // preonly + Jacobi); anything else is refused, not silently changed.
        if (gets("-pc_gamg_type", "agg") != "agg") { std::fprintf(stderr, "main_ksp: only -pc_gamg_type agg\n"); return 1; }
        const char *fixed[][2] = {{"-mg_levels_ksp_type", "richardson"}, {"-mg_levels_ksp_max_it", "1"},
                                  {"-mg_coarse_ksp_type", "preonly"}, {"-mg_levels_sub_pc_type", "jacobi"},
                                  {"-mg_coarse_sub_pc_type", "jacobi"}};
        for (auto &f : fixed)
            if (opt.count(f[0]) && opt[f[0]] != f[1]) {
                std::fprintf(stderr, "main_ksp: %s %s not supported (only %s)\n", f[0], opt[f[0]].c_str(), f[1]);
                return 1;
            }
        gp.threshold = getd("-pc_gamg_threshold", gp.threshold);
        gp.nsmooths = (int32_t)geti("-pc_gamg_agg_nsmooths", gp.nsmooths);
        gp.coarse_eq_limit = (int32_t)geti("-pc_gamg_coarse_eq_limit", gp.coarse_eq_limit);
        gp.max_levels = (int32_t)geti("-pc_mg_levels", gp.max_levels);
        gp.square_graph = (int32_t)geti("-pc_gamg_square_graph", gp.square_graph);
        // this build's extensions: 0 selects the greedy aggregation / the
        // power-iteration emax of rounds 1-4 (PETSc has no such switch)
        gp.coarsen = (int32_t)geti("-aijhip_gamg_coarsen", gp.coarsen);
        gp.eig_ksp = (int32_t)geti("-aijhip_gamg_eig_ksp", gp.eig_ksp);
    }
    const std::string nts = gets("-ksp_norm_type", "preconditioned");
    const int normtype = nts == "unpreconditioned" ? AIJHIP_KSP_NORM_UNPRECONDITIONED
                         : nts == "natural"        ? AIJHIP_KSP_NORM_NATURAL
                         : nts == "none"           ? AIJHIP_KSP_NORM_NONE
                                                   : AIJHIP_KSP_NORM_PRECONDITIONED;

    // -------- createSystem (helper.cpp:22-57): assembled on the device
    // (csrc/poisson.hip), or on the host and uploaded with -aijhip_host_assembly
    const bool host_asm = opt.count("-aijhip_host_assembly") > 0;
    int ndev = 0;
    if (aijhip_device_count(&ndev) != AIJHIP_OK || ndev == 0) {
        std::fprintf(stderr, "main_ksp: no HIP device visible\n");
        return AIJHIP_ERR_NODEVICE;
    }
    const double t_start = now();
    const int64_t m = (int64_t)nx * ny * nz;
    std::vector<double> exact((size_t)m);
    aijhip_mat_t A = nullptr;
    double *d_b = nullptr, *d_x = nullptr;
    HCHK(hipMalloc(&d_b, sizeof(double) * (size_t)m));
    HCHK(hipMalloc(&d_x, sizeof(double) * (size_t)m));
    if (host_asm) {
        int64_t nnz = 0;
        CHK(aijhip_poisson_nnz(nx, ny, nz, 0, nz, &nnz));
        std::vector<int32_t> ai((size_t)m + 1), aj((size_t)nnz);
        std::vector<double> aa((size_t)nnz), rhs((size_t)m);
        double scale = 0.0;
        CHK(aijhip_poisson_fill(nx, ny, nz, 0, nz, 1, ai.data(), aj.data(), aa.data(), &scale));
        CHK(aijhip_poisson_vectors(nx, ny, nz, 0, nz, 1, rhs.data(), exact.data()));
        CHK(aijhip_mat_create(0, (int32_t)m, (int32_t)m, nnz, ai.data(), aj.data(), aa.data(), &A));
        HCHK(hipMemcpy(d_b, rhs.data(), sizeof(double) * (size_t)m, hipMemcpyHostToDevice));
    } else {
        double scale = 0.0;
        CHK(aijhip_mat_create_poisson(0, nx, ny, nz, 0, nz, 1, &scale, &A));
        CHK(aijhip_poisson_vectors_device(nx, ny, nz, 0, nz, 1, d_b, d_x, nullptr));
        HCHK(hipMemcpy(exact.data(), d_x, sizeof(double) * (size_t)m, hipMemcpyDeviceToHost));
    }
    HCHK(hipMemset(d_x, 0, sizeof(double) * (size_t)m));  // VecSet(lhs, 0) (helper.cpp:48)
    HCHK(hipDeviceSynchronize());
    const double t_sys = now();

    // -------- KSPCreate / SetOperators / SetType(CG) / SetFromOptions / SetUp (:92-97)
    aijhip_ksp_t ksp = nullptr;
    CHK(aijhip_ksp_create(A, &ksp));
    CHK(aijhip_ksp_set_tolerances(ksp, getd("-ksp_rtol", 1e-5), getd("-ksp_atol", 1e-50),
                                  getd("-ksp_divtol", 1e5), (int32_t)geti("-ksp_max_it", 10000)));
    CHK(aijhip_ksp_set_pc_type(ksp, pc));
    if (pc == AIJHIP_PC_GAMG) CHK(aijhip_ksp_set_gamg_params(ksp, &gp));
    CHK(aijhip_ksp_set_norm_type(ksp, normtype));
    CHK(aijhip_ksp_set_up(ksp));
    HCHK(hipDeviceSynchronize());
    const double t_solver = now();

    // -------- KSPSolve (:103)
    CHK(aijhip_ksp_solve(ksp, d_b, d_x, nullptr));
    HCHK(hipDeviceSynchronize());
    const double t_solve = now();

    int reason = 0;
    int32_t its = 0;
    double res = 0.0;
    CHK(aijhip_ksp_get_converged_reason(ksp, &reason));
    if (reason < 0) {  // main_ksp.cpp:109-111
        std::fprintf(stderr, "Diverger reason: %d\n", reason);
        return 91;
    }
    CHK(aijhip_ksp_get_iteration_number(ksp, &its));
    CHK(aijhip_ksp_get_residual_norm(ksp, &res));
    // VecAXPY(lhs, -1, exact); VecNorm(lhs, NORM_INFINITY) (:119-121)
    std::vector<double> x((size_t)m);
    HCHK(hipMemcpy(x.data(), d_x, sizeof(double) * (size_t)m, hipMemcpyDeviceToHost));
    double linf = 0.0;
    for (int64_t i = 0; i < m; ++i) linf = std::fmax(linf, std::fabs(x[i] + (-1.0) * exact[i]));

    std::printf("[Nx, Ny, Nz]: [%d, %d, %d]\n" "Number of iterations: %d\n"
                "L2 norm of final residual: %f\n" "Maximum norm of error: %f\n"
                "Time [init, create solver, solve]: [%f, %f, %f]\n",
                nx, ny, nz, its, res, linf, t_sys - t_start, t_solver - t_sys, t_solve - t_solver);
    std::fflush(stdout);

    CHK(aijhip_ksp_destroy(ksp));
    CHK(aijhip_mat_destroy(A));
    hipFree(d_b);
    hipFree(d_x);
    return 0;
}
