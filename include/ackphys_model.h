/* ackphys_model.h -- binary layout of the compiled-model blob passed to ackphys_create().
 *
 * The blob is the compiled form of the reference's MJCF model (the object
 * `mujoco.MjModel.from_xml_path` returns at src/rl/envs/simple_map_spawner.py:37): a fixed
 * header struct `apm_model_t` followed by the mesh arrays it indexes. It is produced by
 * mujoco_playground_amd/model/blob.py (ctypes mirror of this struct) and consumed by
 *   - libackphys.so (HIP product): checks it against the model the kernels were
 *     specialised on (APM hash) and rejects a mismatch;
 *   - oracle/ (CPU restatement, test-only): reads every field.
 * All multi-byte fields are little-endian, naturally aligned, no implicit padding.
 */
#ifndef ACKPHYS_MODEL_H
#define ACKPHYS_MODEL_H

#include <stdint.h>

#define APM_MAGIC 0x4D504841u /* "AHPM" */
#define APM_VERSION 2u

#define APM_MAXBODY 64
#define APM_MAXJNT 8
#define APM_MAXQ 16
#define APM_MAXDOF 16
#define APM_MAXGEOM 64
#define APM_MAXSITE 80
#define APM_MAXSENSOR 96
#define APM_MAXU 4
#define APM_MAXEQ 2
#define APM_MAXMESH 4

/* mjtGeom subset */
#define APM_GEOM_PLANE 0
#define APM_GEOM_SPHERE 2
#define APM_GEOM_CAPSULE 3
#define APM_GEOM_CYLINDER 5
#define APM_GEOM_BOX 6
#define APM_GEOM_MESH 7
/* mjtJoint subset */
#define APM_JNT_FREE 0
#define APM_JNT_HINGE 3
/* sensors */
#define APM_SENS_JOINTPOS 0
#define APM_SENS_JOINTVEL 1
#define APM_SENS_RANGEFINDER 2
/* actuators */
#define APM_ACT_POSITION 0
#define APM_ACT_VELOCITY 1

typedef struct apm_model {
  uint32_t magic, version, nbytes, hdr_bytes;
  int32_t nbody, njnt, nq, nv, ngeom, nsite, nsensor, nsensordata, nu, neq, nmesh;
  int32_t iterations, ls_iterations, pad0;
  int32_t nmeshvert, nmeshface, nhullvert, pad1;
  double timestep, gravity[3], tolerance, impratio, meaninertia;

  /* bodies */
  int32_t body_parentid[APM_MAXBODY], body_rootid[APM_MAXBODY], body_weldid[APM_MAXBODY];
  int32_t body_jntadr[APM_MAXBODY], body_jntnum[APM_MAXBODY];
  int32_t body_dofadr[APM_MAXBODY], body_dofnum[APM_MAXBODY];
  double body_pos[APM_MAXBODY][3], body_quat[APM_MAXBODY][4];
  double body_ipos[APM_MAXBODY][3], body_iquat[APM_MAXBODY][4];
  double body_mass[APM_MAXBODY], body_inertia[APM_MAXBODY][3], body_invweight0[APM_MAXBODY][2];

  /* joints */
  int32_t jnt_type[APM_MAXJNT], jnt_bodyid[APM_MAXJNT], jnt_qposadr[APM_MAXJNT];
  int32_t jnt_dofadr[APM_MAXJNT], jnt_limited[APM_MAXJNT], pad2[APM_MAXJNT];
  double jnt_pos[APM_MAXJNT][3], jnt_axis[APM_MAXJNT][3], jnt_range[APM_MAXJNT][2];
  double jnt_solref[APM_MAXJNT][2], jnt_solimp[APM_MAXJNT][5], jnt_margin[APM_MAXJNT];

  /* dofs */
  int32_t dof_bodyid[APM_MAXDOF], dof_jntid[APM_MAXDOF], dof_parentid[APM_MAXDOF];
  int32_t pad3[APM_MAXDOF];
  double dof_armature[APM_MAXDOF], dof_damping[APM_MAXDOF], dof_frictionloss[APM_MAXDOF];
  double dof_solref[APM_MAXDOF][2], dof_solimp[APM_MAXDOF][5], dof_invweight0[APM_MAXDOF];
  double qpos0[APM_MAXQ];

  /* geoms */
  int32_t geom_type[APM_MAXGEOM], geom_bodyid[APM_MAXGEOM], geom_contype[APM_MAXGEOM];
  int32_t geom_conaffinity[APM_MAXGEOM], geom_condim[APM_MAXGEOM], geom_dataid[APM_MAXGEOM];
  double geom_pos[APM_MAXGEOM][3], geom_quat[APM_MAXGEOM][4], geom_size[APM_MAXGEOM][3];
  double geom_friction[APM_MAXGEOM][3], geom_solref[APM_MAXGEOM][2], geom_solimp[APM_MAXGEOM][5];
  double geom_solmix[APM_MAXGEOM], geom_margin[APM_MAXGEOM], geom_gap[APM_MAXGEOM];
  double geom_rgba[APM_MAXGEOM][4], geom_rbound[APM_MAXGEOM];

  /* sites */
  int32_t site_bodyid[APM_MAXSITE], pad4[2];
  double site_pos[APM_MAXSITE][3], site_quat[APM_MAXSITE][4];

  /* sensors */
  int32_t sensor_type[APM_MAXSENSOR], sensor_objid[APM_MAXSENSOR], sensor_adr[APM_MAXSENSOR];
  int32_t pad5[2];
  double sensor_cutoff[APM_MAXSENSOR];

  /* actuators (transmission: joint, gear[0]) */
  int32_t actuator_type[APM_MAXU], actuator_trnid[APM_MAXU];
  int32_t actuator_ctrllimited[APM_MAXU], actuator_forcelimited[APM_MAXU];
  double actuator_gear[APM_MAXU], actuator_gainprm[APM_MAXU][3], actuator_biasprm[APM_MAXU][3];
  double actuator_ctrlrange[APM_MAXU][2], actuator_forcerange[APM_MAXU][2];

  /* equality constraints (joint type) */
  int32_t eq_obj1id[APM_MAXEQ], eq_obj2id[APM_MAXEQ];
  double eq_polycoef[APM_MAXEQ][5], eq_solref[APM_MAXEQ][2], eq_solimp[APM_MAXEQ][5];

  /* meshes: offsets (in elements) into the trailing arrays */
  int32_t mesh_vertadr[APM_MAXMESH], mesh_vertnum[APM_MAXMESH];
  int32_t mesh_faceadr[APM_MAXMESH], mesh_facenum[APM_MAXMESH];
  int32_t mesh_hulladr[APM_MAXMESH], mesh_hullnum[APM_MAXMESH];
  double mesh_aabb[APM_MAXMESH][6]; /* centre[3], half-size[3] in the mesh (geom) frame */

  /* env spawn point written into the free joint by the reset (scene property; v2: 0 0 0.1,
     simple_map_spawner.py:43) */
  double spawn[3];
} apm_model_t;

/* Trailing arrays, in order, each starting at hdr_bytes + running offset:
 *   float   mesh_vert[nmeshvert][3]   -- all meshes' vertices in their inertial (geom) frame
 *   int32_t mesh_face[nmeshface][3]   -- vertex indices, local to the mesh's vertadr
 *   float   hull_vert[nhullvert][3]   -- convex-hull vertices used for collision
 */

#endif /* ACKPHYS_MODEL_H */
