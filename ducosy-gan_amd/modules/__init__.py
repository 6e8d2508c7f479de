"""MI355X-native mirror of the reference's ``modules`` package (hot path only).

modules.model     — Generator / Discriminator / CBAM / residual blocks (drop-in)
modules.trainer   — loss modules and train_cycle_gan (drop-in)
modules.hip       — C-ABI binding and the fused HIP forward/backward paths
"""
