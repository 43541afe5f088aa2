"""module -- drop-in mirror of the reference's repo-level hot-path modules
(/root/reference/module/{NegativeSampling,loss,submodule,spectral_norm,model,zsl_module}.py),
routed through libmmre_hip.so. The multimodal encoder side (M3AE transformer, RGCN, image/text
reconstruction losses, dataset ingestion) is upstream of the hot path and out of scope."""
