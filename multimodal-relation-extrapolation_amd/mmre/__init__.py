"""mmre -- MI355X-native KG scoring hot path of luisrui/Multimodal-Relation-Extrapolation.

Core package behind the `openke` and `module` drop-in mirrors: the ctypes binding of
libmmre_hip.so (`_lib`), the link-prediction engine (`link`), the fused negative-sampling
loss and sampler (`ns`, `sampler`), the relation generator (`generator`), candidate
rankings (`candidates`), dataset readers (`data`) and the relation-sharded multi-GPU
evaluation (`sharding`).
"""
__version__ = "0.1.0"
