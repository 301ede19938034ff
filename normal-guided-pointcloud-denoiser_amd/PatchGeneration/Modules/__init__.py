"""MI355X-native replacement of PatchGeneration/Modules/Mesh.py (Mesh.updateVertices)."""
