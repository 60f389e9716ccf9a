#ifndef __NET_NET_H__
#define __NET_NET_H__

#include <stdint.h>

#ifndef RT_L2_DATA
#define RT_L2_DATA
#endif

// Network Dimensions
#define NET_F1 16
#define NET_F2 16
#define NET_D 1
#define NET_C 19
#define NET_C_ALIGN 20
#define NET_T 480
#define NET_T_ALIGN 480
#define NET_T8 60
#define NET_T8_ALIGN 60
#define NET_T64 7
#define NET_T64_ALIGN 8
#define NET_N 3
/*
 * Layer 1
 * =======
 * Convolution + BN
 * 
 * Input:  [C, T]
 * Weight: [C, 1]
 * Output: [F2, 1, T]
 */

extern RT_L2_DATA const int32_t net_l1_factor[16];
extern RT_L2_DATA const int32_t net_l1_offset[16];
#define NET_L1_WEIGHT_LEN 19
#define NET_L1_WEIGHT_LEN_ALIGN 20
extern RT_L2_DATA const int8_t net_l1_weight[304];
extern RT_L2_DATA const int8_t net_l1_weight_align[320];
extern RT_L2_DATA const int32_t net_l1_weight_32[304];
/*
 * Layer 2
 * =======
 * Convolution + BN + ReLU + Pooling
 * 
 * Input:  [F2, 1, T]
 * Weight: [F2, 1, 64]
 * Output: [F2, T // 8]
 */

#define NET_L2_PAD_START 31
#define NET_L2_PAD_END 32
#define NET_L2_PAD_INPUT_LEN 543
#define NET_L2_PAD_INPUT_LEN_ALIGN 544
extern RT_L2_DATA const int32_t net_l2_factor[16];
extern RT_L2_DATA const int32_t net_l2_offset[16];
#define NET_L2_WEIGHT_LEN 64
#define NET_L2_WEIGHT_LEN_ALIGN 64
extern RT_L2_DATA const int8_t net_l2_weight[1024];
extern RT_L2_DATA const int8_t net_l2_weight_reverse[1024];
extern RT_L2_DATA const int8_t net_l2_weight_reverse_pad[1024];
/*
 * Layer 3
 * =======
 * Convolution
 * 
 * Input:  [F2, T // 8]
 * Weight: [F2, 16]
 * Output: [F2, T // 8]
 */

#define NET_L3_PAD_START 7
#define NET_L3_PAD_END 8
#define NET_L3_PAD_INPUT_LEN 75
#define NET_L3_PAD_INPUT_LEN_ALIGN 76
#define NET_L3_FACTOR 238
#define NET_L3_WEIGHT_LEN 16
extern RT_L2_DATA const int8_t net_l3_weight[256];
/*
 * Layer 4
 * =======
 * Convolution + BN + ReLU + Pooling
 * 
 * Input:  [F2, T // 8]
 * Weight: [F2, F2]
 * Output: [F2, T // 64]
 */

extern RT_L2_DATA const int32_t net_l4_factor[16];
extern RT_L2_DATA const int32_t net_l4_offset[16];
#define NET_L4_WEIGHT_LEN 16
extern RT_L2_DATA const int8_t net_l4_weight[256];
/*
 * Layer 5
 * =======
 * Linear Layer (without scaling in the end)
 * 
 * Input:  [F2, T // 64]
 * Weight: [N, F2 * (T // 64)]
 * Bias:   [N]
 * Output: [N]
 */

#define NET_L5_FACTOR 562
extern RT_L2_DATA const int8_t net_l5_bias[3];
#define NET_L5_WEIGHT_LEN 128
extern RT_L2_DATA const int8_t net_l5_weight[384];

#endif//__NET_NET_H__
