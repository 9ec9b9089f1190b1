// rt_tables.cpp — embeds the sampler tables (data/ *.u8: g_strata_permutation_sets,
// RT/samplers.cpp:140-397, and the 256spp blue-noise tables, RT/blue_noise_samplers/
// ...256spp.cpp:2-12; extracted by tools/extract_tables.py) and the output dither textures
// (data/noise/LDR_RGB1_*.png, RT/assets.cpp:63-113; tools/extract_noise.py) into the product library.
#ifndef RT_DATA_DIR
#error "RT_DATA_DIR must name the repo's data/ directory"
#endif
#define RT_STR2(x) #x
#define RT_STR(x) RT_STR2(x)
__asm__(
    ".section .rodata\n"
    ".global rt_dev_strata_tab\n"
    ".type rt_dev_strata_tab, @object\n"
    ".balign 64\n"
    "rt_dev_strata_tab:\n"
    ".incbin \"" RT_STR(RT_DATA_DIR) "/strata_permutation_sets.u8\"\n"
    ".size rt_dev_strata_tab, 16384\n"
    ".global rt_dev_bluenoise_tab\n"
    ".type rt_dev_bluenoise_tab, @object\n"
    ".balign 64\n"
    "rt_dev_bluenoise_tab:\n"
    ".incbin \"" RT_STR(RT_DATA_DIR) "/bluenoise_256spp.u8\"\n"
    ".size rt_dev_bluenoise_tab, 327680\n"
    ".global rt_dev_dither_tab\n"
    ".type rt_dev_dither_tab, @object\n"
    ".balign 64\n"
    "rt_dev_dither_tab:\n"
    ".incbin \"" RT_STR(RT_DATA_DIR) "/dither_rgb1_256.u8\"\n"
    ".size rt_dev_dither_tab, 1572864\n"
    ".text\n");
