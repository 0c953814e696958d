bash tools/gpu_steps.sh r06m \
 pmc_b1 900 "bash tools/pmc_mfma.sh r06m_b1" \
 pmc_b64 900 "bash tools/pmc_mfma.sh r06m_b64 --batch 64"
