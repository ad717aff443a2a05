"""Kernel families of the step for the PMC traffic passes (tools/r3/pmc_families.sh)."""
REGEX = {
    "gemm": "conv_gemm_kernel|conv_gemm_glds_kernel|conv_gemm_wreg_kernel|splitk_epilogue_kernel",
    "wgrad": "conv_wgrad_kernel|reduce_partials_kernel",
    "attn": "attn_fwd|attn_bwd|attn_drow",
    "mas": "mas_",  # maximum_path: mas_transpose_kernel + mas_dp(_mw)_kernel + mas_expand_kernel (tools/r5/pmc_mas.sh)
}
