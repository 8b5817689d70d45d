"""Output helpers of the drop-in package (the reference's project/utils)."""
