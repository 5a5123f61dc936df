"""Model families of the hot path, mirroring the reference's model/ package:
constructor signatures, forward() contracts and state_dict keys are the
reference's; the math runs on libmdemi kernels (NHWC inside)."""
