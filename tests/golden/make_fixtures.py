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

out = {"matrices": {"ex1": EX1, "ex2": EX2}, "cases": cases}
path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hand_plans.json")
with open(path, "w") as f:
    json.dump(out, f, indent=1)
print("wrote", path)
