"""Drop-in for the reference package `Pointcloud` (Ruubje/Normal-Guided-Pointcloud-Denoiser), hot path only."""
