# Timing only (unsafe beside other streams): the library's per-device ordering of fused launches
# disabled, to price its event record per call.
edits = [
    ("fc_capi.hip", """  explicit FusedGuard(hipStream_t s) : s_(s) {
    if (capturing(s)) return;""", """  explicit FusedGuard(hipStream_t s) : s_(s) {
    if (s_ || !s_) return;"""),
]
