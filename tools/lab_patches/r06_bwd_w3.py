# film_bwd_fused with three waves per SIMD (__launch_bounds__(256, 3): <= 168 VGPRs) for 1..8-node
# graphs, the two-slice register prefetch (PRE2) off — VERDICT r5 #3's occupancy question, priced
PATCH = [
    ("film_mean_bwd_launch.hpp",
     "if (g.vec == 4 && a.PV == 2 * g.lpc && (pre2 == 1 || (pre2 == 2 && !DXB))) {",
     "if (false) {"),
    ("film_mean_bwd_launch.hpp",
     "      MRP_LAUNCH((mrp::film_bwd_fused<NT, NT, 4, COMPLETE, DXB>), lds);\n    else if (g.vec == 2)",
     "      MRP_LAUNCH((mrp::film_bwd_fused<NT, NT, 4, COMPLETE, DXB, 3>), lds);\n    else if (g.vec == 2)"),
]
