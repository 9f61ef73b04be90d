"""Mirror of the reference package of the same name (HIP-backed)."""
