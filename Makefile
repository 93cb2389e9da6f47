# Builds the C-ABI HIP library for gfx950 in-tree (travels to the GPU box with the snapshot).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC_DIR := animatable_nerf_amd/csrc
SRCS := $(SRC_DIR)/anr_capi.hip $(SRC_DIR)/anr_rays.hip $(SRC_DIR)/anr_mlp.hip $(SRC_DIR)/anr_pack.hip \
        $(SRC_DIR)/anr_gemm.hip $(SRC_DIR)/anr_train.hip $(SRC_DIR)/anr_train_capi.hip \
        $(SRC_DIR)/anr_sdf.hip $(SRC_DIR)/anr_sdf_capi.hip $(SRC_DIR)/anr_mlp_b16.hip \
        $(SRC_DIR)/anr_alpha.hip $(SRC_DIR)/anr_alpha_b16.hip $(SRC_DIR)/anr_mesh.hip $(SRC_DIR)/anr_tgemm.hip $(SRC_DIR)/anr_lgemm.hip \
        $(SRC_DIR)/anr_sdf_train.hip $(SRC_DIR)/anr_resd_b16.hip $(SRC_DIR)/anr_resd_x6.hip $(SRC_DIR)/anr_mlp_x6.hip $(SRC_DIR)/anr_alpha_x6.hip $(SRC_DIR)/anr_tchain.hip
OBJS := $(SRCS:.hip=.o)
DEPS := $(OBJS:.o=.d)
LIB := animatable_nerf_amd/libaninerf_hip.so
CXXFLAGS := -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall -Wno-unused-function -Iinclude

all: $(LIB)

$(SRC_DIR)/%.o: $(SRC_DIR)/%.hip
	$(HIPCC) $(CXXFLAGS) -MMD -MP -c $< -o $@

# the bf16x6 programs without SLP vectorisation: clang pairs the splits' scalar f32 subtractions into
# v_pk_add_f32, which costs more issue cycles beside MFMAs than two v_sub_f32 (same-box A/B round 6:
# sdf_pdf bf16x6 frame 180.0 -> 175.8 ms, k_mlp_x6 cycles -2.4 %, profiles/round6/r8b_*)
$(SRC_DIR)/anr_mlp_x6.o $(SRC_DIR)/anr_resd_x6.o: CXXFLAGS += -fno-slp-vectorize

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@.tmp $(OBJS) && mv -f $@.tmp $@

-include $(DEPS)

resources: $(SRC_DIR)/anr_mlp.hip $(SRC_DIR)/anr_mlp_b16.hip
	$(HIPCC) $(CXXFLAGS) -c $(SRC_DIR)/anr_mlp.hip -o /tmp/anr_mlp_res.o -Rpass-analysis=kernel-resource-usage
	$(HIPCC) $(CXXFLAGS) -c $(SRC_DIR)/anr_mlp_b16.hip -o /tmp/anr_mlp_b16_res.o -Rpass-analysis=kernel-resource-usage

clean:
	rm -f $(OBJS) $(DEPS) $(LIB)

.PHONY: all clean resources

# layer-GEMM timing probe (tools/gemm_probe.hip), run on the GPU box
PROBE := tools/gemm_probe
probe: $(PROBE)
$(PROBE): tools/gemm_probe.hip $(SRC_DIR)/anr_tgemm.hip $(SRC_DIR)/anr_gemm.o $(SRC_DIR)/anr_lgemm.o
	$(HIPCC) $(CXXFLAGS) -c tools/gemm_probe.hip -o tools/gemm_probe.o
	$(HIPCC) $(CXXFLAGS) -DRG_TIMING -c $(SRC_DIR)/anr_tgemm.hip -o tools/gemm_probe_tgemm.o
	$(HIPCC) --offload-arch=$(ARCH) -o $@ tools/gemm_probe.o tools/gemm_probe_tgemm.o $(filter %.o,$^)
# fused-chain timing probe (tools/tchain_probe.hip); TCP_FLAGS selects -D variants of the chain kernels
TCPROBE := tools/tchain_probe
tchain-probe: $(TCPROBE)
$(TCPROBE): tools/tchain_probe.hip $(SRC_DIR)/anr_tchain.hip $(SRC_DIR)/anr_train.h
	$(HIPCC) $(CXXFLAGS) $(TCP_FLAGS) -c $(SRC_DIR)/anr_tchain.hip -o tools/tchain_probe_k.o
	$(HIPCC) $(CXXFLAGS) -c tools/tchain_probe.hip -o tools/tchain_probe.o
	$(HIPCC) --offload-arch=$(ARCH) -o $@ tools/tchain_probe.o tools/tchain_probe_k.o
.PHONY: probe tchain-probe
