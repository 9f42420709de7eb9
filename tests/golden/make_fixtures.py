"""Writes hand_plans.json from hand-derived tables (see README.md).

Each expected array below was derived by reading the cited reference transform and
applying it by hand to the tiny matrix; nothing here is computed by the oracle."""
import json
import os

# ex1: 6x5, 1-based mtx entries; rows 1 and 5 empty (row 5 trailing)
EX1 = {
    "M": 6, "K": 5,
    "entries": [(0, 0), (0, 2), (2, 1), (2, 3), (2, 4), (3, 0),
                (4, 0), (4, 1), (4, 2), (4, 3), (4, 4)],
}
# ex2: 4x40; row0 cols 0..19, row1 empty, row2 cols 0..14, row3 cols 0..4
EX2 = {
    "M": 4, "K": 40,
    "entries": [(0, c) for c in range(20)] + [(2, c) for c in range(15)] + [(3, c) for c in range(5)],
}

G = "GLOBAL_META_"
T = "THREAD_META_"
W = "WARP_META_"
B = "TBLOCK_META_"

cases = []

# thread_total (token_test.cc:1003-1092), sparse_cf = 4
# sort_operator: row nnz [2,0,3,1,5,0] -> order [4,2,0,3,1,5] (get_row_order_by_length.cc)
# remove_empty_row: last sorted row with nnz is 3 -> end_row_index 3
# col pad to multiple of 4 (modify_*_by_col_pad_in_sub_matrix.cc): 5->8, 3->4, 2->4, 1->4
cases.append({
    "matrix": "ex1", "pipeline": "thread_total", "p0": 4,
    "expect": {
        G + "original_nz_row_indices_0": [4, 2, 0, 3, 1, 5],
        G + "end_row_index_0": [3],
        G + "nz_row_indices_0": [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4,
        G + "nz_col_indices_0": [0, 1, 2, 3, 4, 4, 4, 4, 1, 3, 4, 4, 0, 2, 2, 2, 0, 0, 0, 0],
        # vals are entry ids 1..11 (file order); padded entries are 0
        G + "nz_vals_0": [7, 8, 9, 10, 11, 0, 0, 0, 3, 4, 5, 0, 1, 2, 0, 0, 6, 0, 0, 0],
        T + "first_row_indices_0": [0, 1, 2, 3, 4],
        T + "first_nz_indices_0": [0, 8, 12, 16, 20],
    },
})
# block_total (token_test.cc:1458-1514): TBLOCK rows of 1, no sort, no padding
cases.append({
    "matrix": "ex1", "pipeline": "block_total", "p0": 0,
    "expect": {
        B + "first_row_indices_0": [0, 1, 2, 3, 4, 5, 6],
        B + "first_nz_indices_0": [0, 2, 2, 5, 6, 11, 11],
    },
})
# warp_total (token_test.cc:1188-1249)
cases.append({
    "matrix": "ex1", "pipeline": "warp_total", "p0": 0,
    "expect": {
        W + "first_row_indices_0": [0, 1, 2, 3, 4, 5, 6],
        W + "first_nz_indices_0": [0, 2, 2, 5, 6, 11, 11],
    },
})
# tblock rows of 4 + BMW rows of 1 inside BMTBs
cases.append({
    "matrix": "ex1", "pipeline": "tblock_warp_total", "p0": 4,
    "expect": {
        B + "first_row_indices_0": [0, 4, 6],
        B + "first_nz_indices_0": [0, 6, 11],
        B + "first_BMW_indices_0": [0, 4, 6],
        W + "first_row_indices_0": [0, 1, 2, 3, 4, 5, 6],
        W + "first_nz_indices_0": [0, 2, 2, 5, 6, 11, 11],
    },
})
# warp_segment (token_test.cc:1393-1455), VW = 2; 11 nnz padded to 32 (rate 2.9 < 4)
# bitmap: row starts at nz 0,2,5,6 -> 1+4+32+64 = 101
cases.append({
    "matrix": "ex1", "pipeline": "warp_segment", "p0": 2,
    "expect": {
        G + "nz_row_indices_0": [0, 0, 2, 2, 2, 3, 4, 4, 4, 4, 4] + [4] * 21,
        G + "nz_col_indices_0": [0, 2, 1, 3, 4, 0, 0, 1, 2, 3, 4] + [4] * 21,
        G + "BMT_size_of_each_blk_0": [32],
        T + "first_row_indices_0": [0, 6],
        T + "first_nz_indices_0": [0, 32],
        T + "thread_bit_map_0": [101],
        T + "segment_empty_flag_0": [1],
        T + "segment_empty_row_indices_0": [0, 2, 3, 4],
        T + "segment_offset_0": [0],
        T + "segment_ptr_0": [0],
        W + "first_row_indices_0": [0, 6],
        W + "first_nz_indices_0": [0, 32],
        W + "first_BMT_indices_0": [0, 1],
    },
})
# ex2 warp_segment VW=2: 40 nnz -> 64, two BMTs
cases.append({
    "matrix": "ex2", "pipeline": "warp_segment", "p0": 2,
    "expect": {
        T + "first_row_indices_0": [0, 2, 4],
        T + "first_nz_indices_0": [0, 32, 64],
        T + "thread_bit_map_0": [1 + (1 << 20), 8],
        T + "segment_empty_flag_0": [1],
        T + "segment_empty_row_indices_0": [0, 2, 0, 1],
        T + "segment_offset_0": [0, 0],
        T + "segment_ptr_0": [0, 2],
        W + "first_row_indices_0": [0, 4],
        W + "first_nz_indices_0": [0, 64],
        W + "first_BMT_indices_0": [0, 2],
    },
})
# ex2 thread_bit_map VW=2 (THREAD level: no head forcing)
cases.append({
    "matrix": "ex2", "pipeline": "thread_bit_map", "p0": 2,
    "expect": {
        T + "thread_bit_map_0": [1 + (1 << 20), 8],
        T + "segment_empty_flag_0": [1],
        T + "segment_ptr_0": [0, 2],
    },
})
# balanced warp blocking, 16 nnz per BMW (data_transform_common.cc:934-989)
cases.append({
    "matrix": "ex2", "pipeline": "balanced_warp_total", "p0": 16,
    "expect": {
        W + "first_row_indices_0": [0, 1, 4],
        W + "first_nz_indices_0": [0, 20, 40],
    },
})
# ex1 ends with an empty row: the balanced row splitter asserts (:984)
cases.append({"matrix": "ex1", "pipeline": "balanced_warp_total", "p0": 4, "expect_error": True})

# ex3: 4x200; row0 cols 0..99 (100 nnz), row1 empty, row2 cols 0..29, row3 cols 0..63
EX3 = {
    "M": 4, "K": 200,
    "entries": [(0, c) for c in range(100)] + [(2, c) for c in range(30)] + [(3, c) for c in range(64)],
}
# ex4: 3x700; row0 cols 0..599 (600 nnz), row1 cols 0..9, row2 empty (trailing)
EX4 = {
    "M": 3, "K": 700,
    "entries": [(0, c) for c in range(600)] + [(1, c) for c in range(10)],
}

# warp_bit_map (token_test.cc:1250-1315), N=32 cf=1 -> y=32, VW = x = max(128/32, 32) = 32
# col-direction blocking of 64 with padding (fixed_interval_col_direction_..._operator.cc:313-326):
# rows 100 -> 128 (pads repeat col 99, val 0), 30 -> 64, 64 stays, empty row stays empty
# BMT rows (get_begin_rows_of_BMT_after_fixed_blocking_in_col_direction.cc): one per 64-chunk,
# no ending -> [0, 0, 2, 3]; BMT nzs -> [0, 64, 128, 192, 256]; GLOBAL BMT size 64
# merge by 32 (get_begin_*_after_merge_thread.cc): rows [fr[0], fr[last]] = [0, 3]
# relative rows stop at len-1 (last BMT dropped): [0, 0, 2]; relative nzs [0, 64, 128, 192]
# bit_map_of_thread (parent_bit_map_of_thread.cc): bits [1, 0, 1, 1] (+ forced bit 0),
# packed from the group's last BMT down: 0b1101 = 13
cases.append({
    "matrix": "ex3", "pipeline": "warp_bit_map", "p0": 32,
    "expect": {
        G + "nz_row_indices_0": [0] * 128 + [2] * 64 + [3] * 64,
        G + "nz_col_indices_0": list(range(100)) + [99] * 28 + list(range(30)) + [29] * 34 + list(range(64)),
        G + "BMT_size_of_each_blk_0": [64],
        T + "first_row_indices_without_ending_0": [0, 0, 2, 3],
        T + "first_nz_indices_0": [0, 64, 128, 192, 256],
        W + "first_row_indices_0": [0, 3],
        W + "first_nz_indices_0": [0, 256],
        W + "first_row_indices_relative_to_BMW_0": [0, 0, 2],
        T + "first_nz_indices_relative_to_BMW_0": [0, 64, 128, 192],
        W + "first_BMT_indices_0": [0, 4],
        W + "bit_map_of_thread_0": [13],
    },
})
# same matrix, ex4: 600 -> 640 (10 BMTs), 10 -> 64 (1 BMT); rows [0]*10 + [1]
# one 32-BMT group: bits 0 and 10 set -> 1 + 1024
cases.append({
    "matrix": "ex4", "pipeline": "warp_bit_map", "p0": 32,
    "expect": {
        T + "first_row_indices_without_ending_0": [0] * 10 + [1],
        T + "first_nz_indices_0": [64 * i for i in range(11)] + [704],
        W + "first_row_indices_0": [0, 1],
        W + "first_nz_indices_0": [0, 704],
        W + "first_row_indices_relative_to_BMW_0": [0] * 10,
        T + "first_nz_indices_relative_to_BMW_0": [64 * i for i in range(11)],
        W + "first_BMT_indices_0": [0, 11],
        W + "bit_map_of_thread_0": [1025],
    },
})
# tblock_bit_map (token_test.cc:1515-1582), N=32 cf=1 -> x=32, block_size = 256/32 = 8
# ex4: merge by 8 -> rows [fr[0], fr[8], fr[10]] = [0, 0, 1]; nzs [0, 512, 704]; BMTs [0, 8, 11]
# THREAD bit_map_of_thread: row starts [1,0,...,0,1] plus parent heads 0 and 8 (11 is past
# the end) -> [1,0,0,0,0,0,0,0,1,0,1]
# segment_offset.cc (parent_flag true, size 8): zeros between set bits, a run also
# closing at every multiple of 8 -> so[0] = 7, so[8] = 1, others 0
cases.append({
    "matrix": "ex4", "pipeline": "tblock_bit_map", "p0": 8,
    "expect": {
        B + "first_row_indices_0": [0, 0, 1],
        B + "first_nz_indices_0": [0, 512, 704],
        B + "first_BMT_indices_0": [0, 8, 11],
        T + "bit_map_of_thread_0": [1, 0, 0, 0, 0, 0, 0, 0, 1, 0, 1],
        T + "segment_offset_0": [7, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0],
    },
})
# ex3 through tblock_bit_map: one parent of 4 BMTs, bits [1, 0, 1, 1]; so = [1, 0, 0, 0]
cases.append({
    "matrix": "ex3", "pipeline": "tblock_bit_map", "p0": 8,
    "expect": {
        B + "first_row_indices_0": [0, 3],
        B + "first_nz_indices_0": [0, 256],
        B + "first_BMT_indices_0": [0, 4],
        T + "bit_map_of_thread_0": [1, 0, 1, 1],
        T + "segment_offset_0": [1, 0, 0, 0],
    },
})
# ex1 rows of 2..5 nnz padded to 64: 256 / 11 >= PADDING_RATE_UP_BOUND (4): invalid
# (padding_rate_valid_col_direction_with_multiple, data_transform_common.cc:644-690)
cases.append({"matrix": "ex1", "pipeline": "warp_bit_map", "p0": 32, "expect_error": True})

# merge path (get_begin_{rows,nzs}_of_level_after_merge_path.cc:58-95).  ex1 row nnz
# [2,0,3,1,5,0]: non-empty rows 0,2,3,4; count starts at 0 for the first row, then
# +1 per row change: total_path = [2, 6, 8, 14], count 14.  Level starts i = 0,4,8,12:
# first j with total_path[j] > i -> j = 0,1,3,3 -> rows [0,2,4,4], nz = i - j = [0,3,5,9];
# the nz list ends with nnz = 11.  (i = 8 lands on the step that closes row 3.)
cases.append({
    "matrix": "ex1", "pipeline": "merge_path", "p0": 4, "p1": 1,
    "expect": {
        W + "first_row_indices_without_ending_0": [0, 2, 4, 4],
        W + "first_nz_indices_0": [0, 3, 5, 9, 11],
    },
})
# work_size 3 at TBLOCK: i = 0,3,6,9,12 -> j = 0,1,2,3,3 -> rows [0,2,3,4,4], nz [0,2,4,6,9]
cases.append({
    "matrix": "ex1", "pipeline": "merge_path", "p0": 3, "p1": 2,
    "expect": {
        B + "first_row_indices_without_ending_0": [0, 2, 3, 4, 4],
        B + "first_nz_indices_0": [0, 2, 4, 6, 9, 11],
    },
})
# ex2 row nnz [20,0,15,5]: total_path = [20, 36, 42]; work_size 16 at THREAD: i = 0,16,32
# -> j = 0,0,1 -> rows [0,0,2], nz [0,16,31], then 40
cases.append({
    "matrix": "ex2", "pipeline": "merge_path", "p0": 16, "p1": 3,
    "expect": {
        T + "first_row_indices_without_ending_0": [0, 0, 2],
        T + "first_nz_indices_0": [0, 16, 31, 40],
    },
})
# balanced TBLOCK blocking, 16 nnz per BMTB (data_transform_common.cc:934-989 at TBLOCK)
cases.append({
    "matrix": "ex2", "pipeline": "balanced_block_total", "p0": 16,
    "expect": {
        B + "first_row_indices_0": [0, 1, 4],
        B + "first_nz_indices_0": [0, 20, 40],
    },
})
# balanced THREAD blocking, 6 nnz per BMT: rows 0 (20) cut, row1 empty + row2 (15) cut,
# row3 (5) left over -> rows [0,1,3,4], nzs [0,20,35,40]
cases.append({
    "matrix": "ex2", "pipeline": "balanced_thread_total", "p0": 6,
    "expect": {
        T + "first_row_indices_0": [0, 1, 3, 4],
        T + "first_nz_indices_0": [0, 20, 35, 40],
    },
})

# interleaved storage (§8f rank 2, modify_col_indices_by_interlance_storage.cc:45-71) on the
# warp_bit_map plan of ex3: col-direction BMTs of 64 with padding -> rows 100, 0, 30, 64
# padded to 128, 0, 64, 64 (pads repeat the row's last col) -> 4 BMTs of 64:
# b0 = row0 cols 0..63, b1 = row0 cols 64..99 + 28 x 99, b2 = row2 cols 0..29 + 34 x 29,
# b3 = row3 cols 0..63; element i of BMT b moves to b + 4 * i
_bmts = [list(range(64)), list(range(64, 100)) + [99] * 28, list(range(30)) + [29] * 34, list(range(64))]
_rows = [0, 0, 2, 3]
cases.append({
    "matrix": "ex3", "pipeline": "warp_bit_map_interleaved", "p0": 32,
    "expect": {
        G + "BMT_size_of_each_blk_0": [64],
        G + "nz_col_indices_after_interlance_storage_0": [_bmts[b][i] for i in range(64) for b in range(4)],
        G + "nz_row_indices_after_interlance_storage_0": [_rows[b] for i in range(64) for b in range(4)],
    },
})

# interleaving in the tblock_bit_map plan (token_test.cc:1515-1582 + interlance_storage_operator):
# the operator takes its parent level from the DISTRIBUTING operators run before it
# (interlance_storage_operator.cc:12-45); here only the col-direction THREAD blocking ran (the
# TBLOCK level comes later, from the implementing tblock_thread_bit_map_operator), so it
# interleaves at GLOBAL level (modify_col_indices_by_interlance_storage.cc:45-72): spacing =
# the number of BMTs, element i of BMT b -> b + n_BMT * i.  ex3: same arrays as warp_bit_map.
cases.append({
    "matrix": "ex3", "pipeline": "tblock_bit_map_interleaved", "p0": 8,
    "expect": {
        G + "BMT_size_of_each_blk_0": [64],
        G + "nz_col_indices_after_interlance_storage_0": [_bmts[b][i] for i in range(64) for b in range(4)],
        G + "nz_row_indices_after_interlance_storage_0": [_rows[b] for i in range(64) for b in range(4)],
    },
})
# ex4: 11 BMTs of 64 (row0: cols 64b..64b+63 for b < 9, b9 = cols 576..599 + 40 x 599; b10 =
# row1 cols 0..9 + 54 x 9; pads repeat the row's last col) -> element i of BMT b at b + 11 i;
# the TBLOCK parents [0, 8) [8, 11) that tblock_thread_bit_map_operator builds afterwards
# index the interleaved arrays unchanged (first_BMT_indices [0, 8, 11]).
_b4 = [list(range(64 * b, 64 * b + 64)) for b in range(9)] + [list(range(576, 600)) + [599] * 40,
                                                             list(range(10)) + [9] * 54]
_r4 = [0] * 10 + [1]
cases.append({
    "matrix": "ex4", "pipeline": "tblock_bit_map_interleaved", "p0": 8,
    "expect": {
        G + "BMT_size_of_each_blk_0": [64],
        B + "first_BMT_indices_0": [0, 8, 11],
        G + "nz_col_indices_after_interlance_storage_0": [_b4[b][i] for i in range(64) for b in range(11)],
        G + "nz_row_indices_after_interlance_storage_0": [_r4[b] for i in range(64) for b in range(11)],
    },
})

# interleaving under a TBLOCK parent: tblock_col_thread_interleaved on ex1 with BMTBs of 4 rows and
# BMTs of 2.  Rows padded to a multiple of 2 first (pads repeat the row's last col): cols
# [0 2 | 1 3 4 4 | 0 0 | 0 1 2 3 4 4], rows [0 0 2 2 2 2 3 3 4 4 4 4 4 4]; BMTs b0 (0,2) r0,
# b1 (1,3) r2, b2 (4,4) r2, b3 (0,0) r3 | b4 (0,1) b5 (2,3) b6 (4,4) r4; BMTBs rows [0,4) [4,6)
# -> first_BMT [0, 4, 7], sizes [2, 2].  The operator's parent is TBLOCK (a "tblock" distributing
# operator ran before it, interlance_storage_operator.cc:12-45); per parent
# (modify_col_indices_by_interlance_storage.cc:73-118) element i of BMT b -> offset + b + i * n:
# parent 0 (n 4): [b0[0] b1[0] b2[0] b3[0] b0[1] b1[1] b2[1] b3[1]] = [0 1 4 0 2 3 4 0];
# parent 1 (n 3, offset 8): [0 2 4 1 3 4].
cases.append({
    "matrix": "ex1", "pipeline": "tblock_col_thread_interleaved", "p0": 4, "p1": 2,
    "expect": {
        B + "first_BMT_indices_0": [0, 4, 7],
        B + "BMT_size_of_each_blk_0": [2, 2],
        G + "nz_col_indices_after_interlance_storage_0": [0, 1, 4, 0, 2, 3, 4, 0, 0, 2, 4, 1, 3, 4],
        G + "nz_row_indices_after_interlance_storage_0": [0, 2, 2, 3, 0, 2, 2, 3, 4, 4, 4, 4, 4, 4],
    },
})

# the same inside BMWs of 4 rows (warp_col_thread_interleaved): the operator's parent is WARP
cases.append({
    "matrix": "ex1", "pipeline": "warp_col_thread_interleaved", "p0": 4, "p1": 2,
    "expect": {
        W + "first_BMT_indices_0": [0, 4, 7],
        W + "BMT_size_of_each_blk_0": [2, 2],
        G + "nz_col_indices_after_interlance_storage_0": [0, 1, 4, 0, 2, 3, 4, 0, 0, 2, 4, 1, 3, 4],
        G + "nz_row_indices_after_interlance_storage_0": [0, 2, 2, 3, 0, 2, 2, 3, 4, 4, 4, 4, 4, 4],
    },
})

# col padding to the parent's longest row (modify_*_by_col_pad_parent_blk_to_max_row_size.cc,
# padding_with_empty_row false) in tblock_col_thread_maxpad on ex1, BMTBs of 4 rows, BMTs of 2:
# row nnz [2,0,3,1,5,0]; parent rows [0,4) max 3: row0 -> 3 (one pad, col 2), row1 stays empty,
# row3 -> 3 (two pads, col 0); parent [4,6) max 5.  Cols [0 2 2 | 1 3 4 | 0 0 0 | 0 1 2 3 4],
# vals [1 2 0 | 3 4 5 | 6 0 0 | 7 8 9 10 11]; the BMTB level is rebuilt on the padded COO
# (first nz 0, 9, 14); each row cut into chunks of 2: starts 0 2 | 3 5 | 6 8 | 9 11 13, end 14.
cases.append({
    "matrix": "ex1", "pipeline": "tblock_col_thread_maxpad", "p0": 4, "p1": 2,
    "expect": {
        G + "nz_col_indices_0": [0, 2, 2, 1, 3, 4, 0, 0, 0, 0, 1, 2, 3, 4],
        G + "nz_row_indices_0": [0, 0, 0, 2, 2, 2, 3, 3, 3, 4, 4, 4, 4, 4],
        G + "nz_vals_0": [1, 2, 0, 3, 4, 5, 6, 0, 0, 7, 8, 9, 10, 11],
        B + "first_nz_indices_0": [0, 9, 14],
        T + "first_nz_indices_0": [0, 2, 3, 5, 6, 8, 9, 11, 13, 14],
        T + "first_row_indices_without_ending_0": [0, 0, 2, 2, 3, 3, 4, 4, 4],
    },
})

# row-direction BMTs with is_col_padding_with_row_max_size_with_empty_row inside BMTBs of 4 rows
# (tblock_thread_total_maxpad, BMTs of 1 row; fixed_interval_row_direction_thread_blocking_operator
# .cc:369-437 -> modify_*_by_col_pad_parent_blk_to_max_row_size with padding_with_empty_row):
# parent [0,4) max 3, parent [4,6) max 5, EMPTY rows padded too, a pad repeating the last column
# written so far: row0 [0 2 2], row1 [2 2 2], row2 [1 3 4], row3 [0 0 0], row4 [0 1 2 3 4],
# row5 [4 4 4 4 4]; BMTB first nz 0, 12, 22; one BMT per row.
cases.append({
    "matrix": "ex1", "pipeline": "tblock_thread_total_maxpad", "p0": 4, "p1": 1,
    "expect": {
        G + "nz_col_indices_0": [0, 2, 2, 2, 2, 2, 1, 3, 4, 0, 0, 0, 0, 1, 2, 3, 4, 4, 4, 4, 4, 4],
        G + "nz_row_indices_0": [0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 4, 4, 4, 4, 4, 5, 5, 5, 5, 5],
        G + "nz_vals_0": [1, 2, 0, 0, 0, 0, 3, 4, 5, 6, 0, 0, 7, 8, 9, 10, 11, 0, 0, 0, 0, 0],
        B + "first_nz_indices_0": [0, 12, 22],
        T + "first_nz_indices_0": [0, 3, 6, 9, 12, 17, 22],
    },
})

# relative BMW indices (§8f rank 1) on ex1 with BMTBs of 4 rows and BMWs of 2 rows:
# BMTB rows [0,4) and [4,6); BMW starts 0,2 | 4 -> relative 0,2 | 0; row nnz [2,0,3,1,5,0]:
# BMTB 0 nonzeros before each BMW 0, 2 | BMTB 1: 0
cases.append({
    "matrix": "ex1", "pipeline": "tblock_warp_total_relative", "p0": 4, "p1": 2,
    "expect": {
        W + "first_row_indices_relative_to_BMTB_0": [0, 2, 0],
        W + "first_nz_indices_relative_to_BMTB_0": [0, 2, 0],
    },
})

# §8f rank 1, BMTs inside parents (fixed_interval_row_direction_thread_blocking_operator.cc
# :198-480).  ex1 row nnz [2,0,3,1,5,0], BMTBs of 4 rows: [0,4) [4,6), first nz 0 | 6 | 11.
# BMTs of 3 rows start at 0, 3 | 4 (+ row_num 6); relative 0, 3 | 0.  Nz starts: each parent
# opens at its first nz; after rows 0-2 (not the parent's last row) a new BMT at 0+5 = 5;
# BMTB 1 opens at 6, its 2 rows never reach 3 -> [0, 5, 6, 11]; relative 0, 5 | 0;
# BMTs per BMTB 2 | 1 -> first_BMT_indices [0, 2, 3]
TB = "TBLOCK_META_"
cases.append({
    "matrix": "ex1", "pipeline": "tblock_thread_total", "p0": 4, "p1": 3,
    "expect": {
        T + "first_row_indices_0": [0, 3, 4, 6],
        T + "first_row_indices_relative_to_BMTB_0": [0, 3, 0],
        T + "first_nz_indices_0": [0, 5, 6, 11],
        T + "first_nz_indices_relative_to_BMTB_0": [0, 5, 0],
        TB + "first_BMT_indices_0": [0, 2, 3],
    },
})
# the same inside BMWs of 8 rows (one per BMTB here), one row per BMT: a BMT opens after
# every row that does not end its BMW -> nz starts 0, 2, 2, 5 | 6, 11 (+ 11)
cases.append({
    "matrix": "ex1", "pipeline": "tblock_warp_thread_total", "p0": 4, "p1": 1,
    "expect": {
        T + "first_row_indices_0": [0, 1, 2, 3, 4, 5, 6],
        T + "first_row_indices_relative_to_BMW_0": [0, 1, 2, 3, 0, 1],
        T + "first_nz_indices_0": [0, 2, 2, 5, 6, 11, 11],
        T + "first_nz_indices_relative_to_BMW_0": [0, 2, 2, 5, 0, 5],
        W + "first_BMT_indices_0": [0, 4, 6],
    },
})

# balanced BMTs inside row-direction BMTBs (balanced_interval_row_direction_thread_blocking_operator
# .cc:207-249 -> data_transform_common.cc:794-932, get_begin_BMTs_of_specific_parent_after_blocking_
# in_row_direction.cc).  ex1 row nnz [2,0,3,1,5,0], BMTBs of 4 rows [0,4) [4,6) (first nz 0, 6, 11),
# 3 nnz per BMT: a BMT closes after the row where the running count reaches 3, unless that row ends
# the parent.  BMTB 0: rows 0 (2), 1 (2), 2 (5 >= 3) -> cut before row 3 at nz 5; BMTB 1: row 4
# (5 >= 3, not the last row) -> cut before row 5 at nz 6 + 5 = 11.  Rows close with row_num 6, nzs
# with the last parent nz 11.  BMTs per BMTB 2 | 2.
cases.append({
    "matrix": "ex1", "pipeline": "tblock_balanced_thread_total", "p0": 4, "p1": 3,
    "expect": {
        T + "first_row_indices_0": [0, 3, 4, 5, 6],
        T + "first_row_indices_relative_to_BMTB_0": [0, 3, 0, 1],
        T + "first_nz_indices_0": [0, 5, 6, 11, 11],
        T + "first_nz_indices_relative_to_BMTB_0": [0, 5, 0, 5],
        B + "first_BMT_indices_0": [0, 2, 4],
    },
})
# ex2 row nnz [20,0,15,5], BMTBs of 2 rows [0,2) [2,4) (first nz 0, 20, 40), 6 nnz per BMT: row 0
# (20) and row 2 (15) each close a BMT; the empty row 1 and row 3 end their parents.
cases.append({
    "matrix": "ex2", "pipeline": "tblock_balanced_thread_total", "p0": 2, "p1": 6,
    "expect": {
        T + "first_row_indices_0": [0, 1, 2, 3, 4],
        T + "first_row_indices_relative_to_BMTB_0": [0, 1, 0, 1],
        T + "first_nz_indices_0": [0, 20, 20, 35, 40],
        T + "first_nz_indices_relative_to_BMTB_0": [0, 20, 0, 15],
        B + "first_BMT_indices_0": [0, 2, 4],
    },
})

# one-row BMTs inside BMTBs with every row padded to a multiple of the column count
# (fixed_interval_row_direction_thread_blocking_operator.cc:272-310 with is_col_padding_with_col_size:
# modify_*_by_col_pad_in_sub_matrix, then the BMTB operator rerun on the padded COO).  ex1 with
# col_size 2: row nnz [2,0,3,1,5,0] -> [2,0,4,2,6,0], pads repeat the row's last column with value
# 0; BMTBs of 4 rows: first nz 0, 8, 14; one BMT per row (empty rows too).
cases.append({
    "matrix": "ex1", "pipeline": "tblock_thread_total_colpad", "p0": 4, "p1": 2,
    "expect": {
        G + "nz_col_indices_0": [0, 2, 1, 3, 4, 4, 0, 0, 0, 1, 2, 3, 4, 4],
        G + "nz_row_indices_0": [0, 0, 2, 2, 2, 2, 3, 3, 4, 4, 4, 4, 4, 4],
        G + "nz_vals_0": [1, 2, 3, 4, 5, 0, 6, 0, 7, 8, 9, 10, 11, 0],
        B + "first_nz_indices_0": [0, 8, 14],
        T + "first_row_indices_0": [0, 1, 2, 3, 4, 5, 6],
        T + "first_nz_indices_0": [0, 2, 2, 6, 8, 14, 14],
        T + "first_row_indices_relative_to_BMTB_0": [0, 1, 2, 3, 0, 1],
        T + "first_nz_indices_relative_to_BMTB_0": [0, 2, 2, 6, 0, 6],
        B + "first_BMT_indices_0": [0, 4, 6],
    },
})

# nnz-direction BMTBs (fixed_interval_nnz_direction_tblock_blocking_operator.cc:95-147): the COO is
# padded to a multiple of nnz_per_BMTB by repeating the last entry's row and column with value 0
# (modify_*_by_nnz_pad.cc), BMTB i starts at nz i * p0 and at that entry's row, the row list closes
# with row_num (get_begin_{rows,nzs}_of_BMTB_after_fixed_blocking_in_nnz_direction.cc).  Then 32-nnz
# BMTs inside with indices relative to the BMTB (fixed_interval_nnz_direction_thread_blocking_operator
# + get_begin_{rows,nzs}_of_BMT_after_fixed_blocking_in_nnz_direction_relative_to_BMTB.cc) and the
# thread bitmap (a bit per row start inside each BMT).
# ex2: 40 nnz -> 64 (24 pads of row 3, col 4); rows of entries 0..19 = 0, 20..34 = 2, 35..63 = 3.
cases.append({
    "matrix": "ex2", "pipeline": "nnz_tblock_bitmap", "p0": 64,
    "expect": {
        G + "nz_row_indices_0": [0] * 20 + [2] * 15 + [3] * 29,
        G + "nz_col_indices_0": list(range(20)) + list(range(15)) + list(range(5)) + [4] * 24,
        B + "first_row_indices_0": [0, 4],
        B + "first_nz_indices_0": [0, 64],
        T + "first_row_indices_0": [0, 2, 4],
        T + "first_nz_indices_0": [0, 32, 64],
        T + "first_row_indices_relative_to_BMTB_0": [0, 2],
        T + "first_nz_indices_relative_to_BMTB_0": [0, 32],
        B + "first_BMT_indices_0": [0, 2],
        T + "thread_bit_map_0": [1 + (1 << 20), 8],
    },
})
# the same with BMTBs of 32 nnz: one BMT per BMTB, BMTB 1 opens mid-row 2
cases.append({
    "matrix": "ex2", "pipeline": "nnz_tblock_bitmap", "p0": 32,
    "expect": {
        B + "first_row_indices_0": [0, 2, 4],
        B + "first_nz_indices_0": [0, 32, 64],
        T + "first_row_indices_0": [0, 2, 4],
        T + "first_row_indices_relative_to_BMTB_0": [0, 0],
        T + "first_nz_indices_relative_to_BMTB_0": [0, 0],
        B + "first_BMT_indices_0": [0, 1, 2],
        T + "thread_bit_map_0": [1 + (1 << 20), 8],
    },
})
# nnz-direction BMWs of 128 inside BMTBs of 256 (fixed_interval_nnz_direction_warp_blocking_operator,
# relative to the BMTB) and 32-nnz BMTs inside the BMWs (relative to the BMW).  ex4: 610 nnz -> 768
# (158 pads of row 1, col 9); entries 0..599 row 0, 600..767 row 1; row_num 3.
# BMTBs at nz 0, 256, 512 all open in row 0.  BMWs at nz 0, 128, ..., 640: rows 0 x5, then 1;
# relative to their BMTB (first row 0): the same.  BMTs every 32 nz: rows 0 for nz 0..576 (19
# BMTs), 1 for nz 608..736 (5); relative to the BMW: the BMT at 608 lies in BMW 4 (first row 0) -> 1,
# those at 640.. in BMW 5 (first row 1) -> 0.  Row starts: nz 0 (BMT 0, bit 0), nz 600 (BMT 18,
# bit 24).
cases.append({
    "matrix": "ex4", "pipeline": "nnz_tblock_warp_bitmap", "p0": 256, "p1": 128,
    "expect": {
        B + "first_row_indices_0": [0, 0, 0, 3],
        B + "first_nz_indices_0": [0, 256, 512, 768],
        W + "first_row_indices_0": [0, 0, 0, 0, 0, 1, 3],
        W + "first_nz_indices_0": [0, 128, 256, 384, 512, 640, 768],
        W + "first_row_indices_relative_to_BMTB_0": [0, 0, 0, 0, 0, 1],
        W + "first_nz_indices_relative_to_BMTB_0": [0, 128, 0, 128, 0, 128],
        B + "first_BMW_indices_0": [0, 2, 4, 6],
        T + "first_row_indices_0": [0] * 19 + [1] * 5 + [3],
        T + "first_nz_indices_0": [32 * i for i in range(25)],
        T + "first_row_indices_relative_to_BMW_0": [0] * 19 + [1] + [0] * 4,
        T + "first_nz_indices_relative_to_BMW_0": [0, 32, 64, 96] * 6,
        W + "first_BMT_indices_0": [0, 4, 8, 12, 16, 20, 24],
        T + "thread_bit_map_0": [1] + [0] * 17 + [1 << 24] + [0] * 5,
    },
})

out = {"matrices": {"ex1": EX1, "ex2": EX2, "ex3": EX3, "ex4": EX4}, "cases": cases}
path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hand_plans.json")
with open(path, "w") as f:
    json.dump(out, f, indent=1)
print("wrote", path)
