/*
 * pcl_oracle.h -- CPU restatement of the point-cloud emit of point_cloud/src/pcd_write.cpp
 * (convertCVMatToPCL + pcl::VoxelGrid<PointXYZRGB>).  TEST INFRASTRUCTURE ONLY; see pcl_oracle.c.
 * Points are 16-byte PointXYZRGB records {x, y, z, rgba bits} as savePCDFileBinary writes them.
 */
#ifndef SDR_PCL_ORACLE_H
#define SDR_PCL_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* xyz: float [H][W][3]; bgr: u8 [H][W][3] or NULL; out: float [H*W][4] */
void orc_xyz_to_cloud(const float* xyz, const uint8_t* bgr, int W, int H, float* out);
/* returns 1 for PCL's int32-overflow passthrough (out = input), else 0; *count = output points */
int orc_voxel_grid(const float* pts, int n, float lx, float ly, float lz, float* out, int* count);

#ifdef __cplusplus
}
#endif
#endif
