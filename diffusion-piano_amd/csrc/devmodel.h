// Device-side model tables for the pianosim kernels (float, flattened, plus the
// topology tables the wave-cooperative phases iterate over). Built on the host from a
// ps_model_desc by build_dev_model() in pianosim.hip.
#pragma once
#include <stdint.h>

#include "../../include/pianosim.h"

namespace ps {

constexpr int NK = PS_NKEY;
constexpr int NH = PS_NHAND;
constexpr int NB = PS_HAND_NBODY;
constexpr int ND = PS_HAND_NDOF;
constexpr int NG = PS_HAND_NGEOM;
constexpr int NA = PS_HAND_NACT;
constexpr int NV = PS_NV;
constexpr int NU = PS_NU;
constexpr int NBT = NH * NB;   // 50 hand bodies
constexpr int NDT = NH * ND;   // 52 hand dofs (lane l <-> hand dof l)
constexpr int NGT = NH * NG;   // 40 capsules
constexpr int NX = PS_HAND_NXGEOM;
constexpr int NXT = NH * NX;   // 24 box / hull colliders: lanes NGT .. NGT + NXT - 1
constexpr int NCOLL = NGT + NXT;  // global collider ids: capsules, then the extra colliders
static_assert(NCOLL <= 64, "one lane per collider");
constexpr int NTT = NH * PS_HAND_NTENDON;
constexpr int MAXDEP = 9;      // ancestor list length (self + up to 8 ancestors)
constexpr int MAXLEV = 8;      // body tree levels
constexpr int MAXCHILD = 5;
constexpr int MAXCON = 24;     // per-env contact capacity of the GPU workspace
constexpr int KEYLANE = 52;    // lane that carries a row's key-dof entry
// Contact direction rows J are stored compressed: a contact touches the ancestor chains of at
// most two hand bodies (<= 2 * MAXDEP hand dofs, in support-mask bit order) plus one key.
constexpr int YS = 20;         // row stride: 18 hand slots, [YKEY] = key entry, 1 pad
constexpr int YKEY = 19;
constexpr int NTRI = MAXDEP * (MAXDEP - 1) / 2;  // (a,b) pairs 1<=a<=b<=8
constexpr int NKB = 64;        // key-range buckets along y
constexpr int KGEO = 16;       // floats per key collision record
// hull support cells: the direction sphere as a cube map of 6 faces x XCG x XCG cells; per hull
// and cell the vertices that can be the support of a direction in the cell (DevModel::x_cell)
constexpr int XCG = 4;
constexpr int XNCELL = 6 * XCG * XCG;
constexpr int XCV = 8;  // candidates per cell in the support-cell vertex table (DevModel::x_cellv)

struct DevModel {
  float timestep;
  int nsub;
  float grav[3];
  float hgrav[3];  // gravity the hand bodies feel: grav (1 - hand_gravcomp)
  // keys
  float key_pos[NK][3], key_half[NK][3], key_anchor[NK][3];
  float key_mass[NK], key_Minv[NK], key_Mhinv[NK], key_damp[NK], key_stiff[NK], key_sref[NK];
  float key_lo[NK], key_hi[NK], key_ylo[NK], key_yhi[NK], key_binv[NK], key_dinv[NK];
  float base_pos[3], base_half[3];
  float pc_solref[2], pc_solimp[5], pc_fric;
  float hc_solref[2], hc_solimp[5], hc_fric;
  float lim_solref[2], lim_solimp[5];
  float fr_solref[2], fr_solimp[5];   // solreffriction / solimpfriction (friction-loss rows)
  // hand bodies, global index B = h*NB + b
  int body_parent[NBT];
  float body_pos[NBT][3], body_Q[NBT][9], body_mass[NBT], body_ipos[NBT][3], body_I[NBT][6];
  float body_binv[NBT];
  int body_dof[NBT], body_ndof[NBT];
  uint64_t body_pathmask[NBT];  // bit l: hand dof l acts on the body
  int nlev, lev_start[MAXLEV + 1], lev_body[NBT];
  int body_nchild[NBT], body_child[NBT][MAXCHILD];
  // hand dofs, global index g = h*ND + j
  int dof_body[NDT], dof_type[NDT], dof_limited[NDT];
  float dof_axis[NDT][3], dof_lo[NDT], dof_hi[NDT], dof_damp[NDT], dof_arm[NDT], dof_dinv[NDT];
  float dof_floss[NDT];      // frictionloss (0: no friction-loss row)
  int dof_depth[NDT], dof_anc[NDT][MAXDEP];
  uint64_t dof_ancmask[NDT];
  uint64_t dof_descmask[NDT];  // bit g: hand dof g is a proper descendant
  int dof_ndesc[NDT], dof_desc[NDT][ND];
  int ndepth, dep_start[MAXDEP + 1], dep_dof[NDT];
  int dof_act[NDT];          // actuator driving the dof (global index) or -1
  float dof_act_coef[NDT];
  int obs_dof[NDT];          // joints_pos order -> global dof (n_obsj entries: rh then lh)
  int n_obsj;
  uint64_t dof_lockmask;     // bit g: hand dof g is locked (a joint the reference's hand lacks)
  int act_src[NU];           // column of actuator a in the caller's action row (-1: absent)
  int n_action;              // action row width (the last column: sustain)
  // actuators, global a = h*NA + a
  int act_kind[NU], act_dof0[NU], act_dof1[NU], act_flim[NU];
  float act_c0[NU], act_c1[NU], act_kp[NU], act_clo[NU], act_chi[NU], act_flo[NU], act_fhi[NU];
  // colliders: the body of every collider (capsules, then extras); capsule geometry
  int geom_body[NCOLL];
  uint64_t geom_pathmask[NCOLL];  // body_pathmask / body_binv of geom_body: one load, not two
  float geom_binv[NCOLL];
  float geom_pos[NGT][3], geom_axis[NGT][3], geom_hl[NGT], geom_r[NGT];
  int root_geom_count;
  // fingertip sites
  int site_body[NH * PS_NFINGER];
  float site_pos[NH * PS_NFINGER][3];
  // capsule-capsule pairs
  int npairs;
  int pair[PS_MAX_CAPPAIRS][2];
  // extra (box / hull) colliders, global extra index e = h*NX + i (lane NGT + e)
  int nx;                      // extra colliders in use (0: the extra passes are skipped)
  int x_type[NXT];             // PS_GEOM_NONE / BOX / HULL
  float x_pos[NXT][3], x_Q[NXT][9], x_hs[NXT][3], x_rb[NXT];
  int x_v0[NXT], x_nv[NXT];    // hull vertices [x_v0, x_v0 + x_nv) of hull_v
  float x_ec[NXT][8];          // hull: an enclosing capsule in the geom frame (p0, p1, radius, pad)
  // hull: per support cell (hull_cell) the bit mask of the vertices (hull-relative index) that
  // can be a support of a direction in the cell; the others are beaten by one vertex by a margin
  // over the whole (grown) cell, so the fp32 scan over the mask finds the same first maximal
  // vertex as the scan over all of them
  uint64_t x_cell[NXT][XNCELL];
  // hull: the same candidates' fp32 coordinates per cell (ascending vertex order, padded with the
  // last one; cell XNCELL = vertex 0, the zero direction's): one 128-byte read per support search
  // instead of the mask read and then the vertex reads. x_cellv_ok = 0 when a cell holds more
  // than XCV candidates (the mask scan is used)
  alignas(16) float x_cellv[NXT][XNCELL + 1][XCV][4];
  int x_cellv_ok[NXT];
  int nxpairs;                 // hand-hand pairs with an extra collider: a | b << 8
  int nxpairs_same;            // leading ones within one hand (the rest cross hands)
  int xpair[PS_MAX_XPAIRS];
  alignas(16) float hull_v[NH * PS_HAND_HULLVERT][4];  // geom frame (w unused)
  // triangular (a,b) table for the LDL update
  int tri_a[NTRI + 8], tri_b[NTRI + 8];
  // v2 lane-owned topology (packed, loaded into registers once per launch)
  int body_level[NBT];
  int body_child_pack[NBT];   // up to 5 children, 6 bits each (child global body index)
  int dof_anc_pack[NDT][3];   // anc[1..8] as bytes (255 = none): [0]=anc1..4, [1]=anc5..8
  float key_top_zmax;         // max over keys of (z + half_z) + 0.02 : capsule z prefilter
  float piano_xmin, piano_xmax;  // x extent of keys (+0.02) and base for the x prefilter
  // key range of a y interval: NKB buckets over the keys' y extent, kb_first[b] = first key
  // with yhi >= bucket start, kb_end[b] = first key with ylo > bucket end (conservative)
  float kb_y0, kb_inv;
  uint8_t kb_first[NKB], kb_end[NKB];
  int npairs_same;            // leading capsule pairs within one hand (the rest cross hands)
  // per-key collision record, staged into LDS by collide2: pos(3) half(3) anchor(3), then the
  // conservative AABB of the key box over its joint range: xlo xhi ylo yhi ztop, pad
  alignas(16) float key_geo[NK][KGEO];
};

}  // namespace ps
