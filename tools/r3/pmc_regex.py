"""Kernel families of the step for the PMC traffic passes (tools/r3/pmc_families.sh)."""
REGEX = {
    "gemm": "conv_gemm_kernel|conv_gemm_glds_kernel|splitk_epilogue_kernel",
    "wgrad": "conv_wgrad_kernel|reduce_partials_kernel",
    "attn": "attn_fwd_kernel|attn_bwd_dq_kernel|attn_bwd_dkv_kernel|attn_fwd_short_kernel|attn_bwd_dq_short_kernel|attn_bwd_dkv_short_kernel",
}
