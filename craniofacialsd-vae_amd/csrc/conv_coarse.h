// Coarse-level SpiralConv launchers (spiral_conv_coarse.hip).
#pragma once
#include "cfsd_common.h"

namespace cfsd {
struct DwLatArgs;  // conv_lat.h
namespace coarse {

// Layers below this many rows (batch x output vertices) take the slot-group
// kernels: the coarse levels of the hierarchy, where one wave per tile and
// all nine slots cannot fill the chip.
constexpr long kMaxRows = 24576;
// "few-tile" layers (<= ~2 16-row tiles per CU): the fused up-sampling and the
// slot-group data gradient apply below this many tiles
constexpr long kMaxTilesFew = 512;

struct FwdKsArgs {
  const float* x;       // input rows; UP: the coarse tensor [batch, n_coarse, CIN] (batch-major)
  const int* idx;       // spiral [rows][9] (indices into the input level)
  const float* w;       // [COUT][9 CIN]
  const float* bias;    // [COUT] or null
  float* y;             // [batch, rows, COUT] in layout yvm
  float* yup;           // UP: the up-sampled input [batch, rows, CIN] (written), or null
  const int* up_col;    // UP (conv_fwd_pt): composite table [rows][9][3], the 3 coarse columns of the
                        // up-sampled row at spiral position (r, s) (topology.up_comp), else null
  const float* up_val;  // UP: the matching [rows][9][3] values
  int vsrc, rows, batch, n_coarse;
  long total_rows;      // batch * rows
  int xvm, yvm, elu;
};

struct DxKsArgs {
  const float* dpre;      // [batch, rows, COUT] batch-major
  const int* inv_ptr;     // inverse spiral CSR (vsrc*9 + 1)
  const int* inv_row;
  const int4* inv_head;   // first four rows of every (u, s) list, -1 absent
  const float* w;         // [COUT][9 CIN]
  const float* elu_y;     // [batch, vsrc, CIN] ELU output (dx *= ELU'), or null
  float* dx;              // [batch, vsrc, CIN]
  int vsrc, rows, batch;
  long total_rows;        // batch * vsrc (dx rows)
};

bool fwd_ks_enabled(long total_rows, int cin, int cout);
bool fwd_up_supported(long total_rows, int cin, int cout);
int launch_fwd_ks(const FwdKsArgs& a, int cin, int cout, hipStream_t st);
bool dx_ks_enabled(long total_src_rows, int cin, int cout);
int launch_dx_ks(const DxKsArgs& a, int cin, int cout, hipStream_t st);
// dx (as launch_dx_ks) + dW slabs (conv_dw_lat_body, dw_tasks = chunks x units) in one launch
int launch_bwd_ks_pair(const DxKsArgs& a, const DwLatArgs& d, long dw_tasks, int cin, int cout, hipStream_t st);

}  // namespace coarse
}  // namespace cfsd
