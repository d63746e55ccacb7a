from mjlab_amd.scene.scene import Scene, SceneCfg, TerrainImporter, TerrainImporterCfg

__all__ = ["Scene", "SceneCfg", "TerrainImporter", "TerrainImporterCfg"]
