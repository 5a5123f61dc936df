"""Mirror of the reference's utils/ surface that sits on the hot path:
dist_utils (metric collectives, RCCL backend), depth_utils (eval crop + the
9 depth metrics, with a GPU reduction), common_utils.parse (JSON configs)."""
