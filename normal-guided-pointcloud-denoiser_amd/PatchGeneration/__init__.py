"""Drop-in for the reference package `PatchGeneration` (mesh vertex update only)."""
