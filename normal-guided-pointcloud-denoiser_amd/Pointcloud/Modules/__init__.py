"""MI355X-native replacements of Pointcloud/Modules (hot path: selection, tensor voting, position updates)."""
