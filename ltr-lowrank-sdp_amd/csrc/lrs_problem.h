// lrs_problem.h -- host-side problem model: SDPA reader, presolve into the
// device formats of lrs_device.h, and upload.
#pragma once
#include <string>
#include <vector>

#include "lrs_device.h"

namespace lrs {

struct HostEntry {      // one merged coefficient entry of constraint `con` in a cone
    int con;            // 0-based constraint index
    int slot;           // local slot in the cone pattern
    double a;           // raw value (lower triangle)
    bool diag;
    bool owned = true;  // sharded solve: the slot's lower row is this shard's (the entry counts in A(.))
};

struct HostCone {
    int n = 0;
    int nnzRows = 0;                     // constraints with a nonzero coefficient (statNnz)
    bool denseCoeff = false;             // some coefficient >10% fill (reference dense path)
    std::vector<int> prow, pcol;         // pattern, row-major lower (col <= row)
    std::vector<double> Craw;            // C per slot (0 where absent)
    std::vector<char> Chas;              // C has an entry at this slot
    std::vector<HostEntry> ent;          // constraint entries sorted by (con, slot)
    std::vector<int> adj_ptr, adj_low, adj_col, adj_slot;   // symmetric adjacency
    double cNrm1 = 0, cNrm2sq = 0, cNrmInf = 0;
    // dense objective: C kept as a full n x n row-major matrix for the
    // FP64 matrix cores, out of the slot pattern (which then holds the constraints only)
    bool dense_c = false;
    std::vector<double> Cfull;
    // constant objective C = c_alpha J (every entry of the block equal, e.g. Lovász theta's -J):
    // the dense path's products without the matrix, C X = c_alpha 1 (1^T X)
    bool const_c = false;
    double c_alpha = 0.0;
    // sharded solve: this shard's owned local rows [own0, own1) (own1 < 0: every row, unsharded).
    // The 2-D tiles of the stage kernels then cover the owned rows only.
    int own0 = 0, own1 = -1;
    // the LP block (last block of negative size in SDPA) as the diagonal cone at rank 1
    // (build_problem): its columns are the rows, every slot (j, j)
    bool lp = false;
    std::vector<double> lp_nrm2;   // LP block: per column ||a_j||_2^2 of its raw entries
    long lp_dense_dropped = 0;     // LP block: constraint entries of LP_COEFF_DENSE columns (dropped)
};
// Dense-objective policy: LRS_DENSE_C=0 never, =1 every cone with objective entries, unset:
// cones with n >= kDenseCMinN whose C fills >= 1/4 of the lower triangle (measured: the dense
// path is 0.86x the slot path at n = 500, 2.2x at n = 2000, scripts/c5b_probe.py).
constexpr int kDenseCMinN = 1024;
// Constant-objective policy: a block whose C has all n (n + 1) / 2 entries equal can take the
// rank-one products (any n >= 2).  LRS_CONST_C=1 every such block, =0 none; unset: only when
// the whole problem fits the single-workgroup inner loop at every rank the solve can reach
// (every cone's C constant or absent; R and D of all cones at the widest layout of
// sqrt(2 nnzRows) + 1 columns plus the constraint pattern within kSmallLdsBudget of LDS -- or,
// every constraint inside one cone and at most kSmallAutoMaxCones cones, each cone's within it
// (a workgroup a cone); one row layout for every cone; at most kSmallAutoMaxConst constant cones and, unless LRS_SMALL=1,
// kSmallAutoMaxGlobal multi-slot constraints; not under LRS_SMALL=0) --
// that loop needs the constant form (the slot form's n (n + 1) / 2 objective slots do not fit
// one CU), while the multi-launch iteration runs faster on the slot form (theta3: 44 us vs
// 64 us per iteration, profiles/r03e_theta_const.md).
constexpr int kConstCMinN = 2;
constexpr long kSmallLdsBudget = 136 * 1024;   // = lrs_kernels.hip kSmallMaxDynLds
constexpr int kSmallAutoMaxGlobal = 16;        // = lrs_solver.cpp kSmallMaxGlobal
constexpr int kSmallAutoMaxConst = 4;          // = lrs_kernels.hip kSmallMaxConst
constexpr int kSmallAutoMaxCones = 8;          // = lrs_kernels.hip kSmallMaxWg (one workgroup per cone)

struct HostProblem {
    int m = 0, K = 0, nLp = 0;   // K counts the LP cone (the last one) when nLp > 0
    std::vector<double> b;
    std::vector<HostCone> cones;
    long nEntries = 0;
    std::vector<char> force_glob;        // sharded solve: constraints kept on the multi-slot path
    double bNrm1 = 0, bNrm2 = 0, bNrmInf = 0;
    double cNrm1 = 0, cNrm2 = 0, cNrmInf = 0;
};

// SDPA reader with the semantics of io/lorads_file_io.c:59-455
// (C = -F0, |v| < 1e-12 dropped, (i,j) swapped into the lower triangle).
bool read_sdpa(const std::string &path, HostProblem &hp, std::string &err);

// Same presolve from in-memory SDPA-style entries (1-based block/row/col, con 0 = F0).
bool build_problem_coo(int m, int nblk, const int *dims, const double *b, long nnz, const int *con,
                       const int *blk, const int *row, const int *col, const double *val, HostProblem &hp,
                       std::string &err);

// Sharded solve: the rows of every cone split into `world` contiguous
// blocks balanced by adjacency entries (a multi-block problem: each block split alike).  Shard `rank` owns rows
// [bounds[rank], bounds[rank+1]); its local problem holds the owned rows plus the halo
// (the other shards' rows its rows are adjacent to), numbered in global order, the slots
// with at least one owned endpoint, and every constraint with an entry on such a slot.
// A slot -- and each constraint entry on it -- belongs to the shard owning its lower row
// (the row whose kernels evaluate it).  A constraint present on several shards is
// "shared": every holder keeps it on the multi-slot path, sums its owned entries, and the
// partial sums meet in an all-reduce of the shared constraints (primary holder: the
// lowest rank, which alone counts it in sums over constraints).  Norms and rank
// statistics stay the global ones.
struct ShardConePlan {
    int n_global = 0;
    std::vector<int> bounds;                 // [world + 1] global row partition of this cone
    std::vector<int> gid;                    // local row -> global row
    int row0 = 0, nown = 0;                  // owned rows: local [row0, row0 + nown)
    std::vector<int> send_ptr, send_rows;    // rows sent to each peer: local ids, grouped by peer
    std::vector<int> recv_start, recv_cnt;   // halo rows from each peer: local first row, count
};
struct ShardPlan {
    int world = 1, rank = 0;
    std::vector<ShardConePlan> cones;        // every cone's rows split the same way
    std::vector<int> con_gid;                // local constraint -> global constraint
    std::vector<int> shared_gid;             // shared constraints, ascending global id (same on every shard)
    std::vector<int> shared_lid;             // per shared constraint: its local id here, or -1
    std::vector<char> primary;               // per local constraint: this shard counts it in sums
};
bool shard_problem(const HostProblem &g, int world, int rank, HostProblem &out, ShardPlan &plan, std::string &err);

// Device upload of everything that does not depend on the rank.
bool upload_problem(const HostProblem &hp, DevProblem &dp, std::string &err);
void free_problem(DevProblem &dp);

}  // namespace lrs
