# models package: drop-in mirror of the reference's project/models
# (encoders / fusion / model_wrapper) running on MI355X HIP kernels.
