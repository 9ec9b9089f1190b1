/* oracle_tables.c — embeds the sampler tables (data/ *.u8, extracted from the
 * reference by tools/extract_tables.py) into liboracle.so.  TEST INFRASTRUCTURE. */
#ifndef RT_DATA_DIR
#error "RT_DATA_DIR must name the repo's data/ directory"
#endif
#define RT_STR2(x) #x
#define RT_STR(x) RT_STR2(x)
__asm__(
    ".section .rodata\n"
    ".global rt_strata_permutation_sets\n"
    ".type rt_strata_permutation_sets, @object\n"
    ".balign 64\n"
    "rt_strata_permutation_sets:\n"
    ".incbin \"" RT_STR(RT_DATA_DIR) "/strata_permutation_sets.u8\"\n"
    ".size rt_strata_permutation_sets, 16384\n"
    ".global rt_bluenoise_256spp\n"
    ".type rt_bluenoise_256spp, @object\n"
    ".balign 64\n"
    "rt_bluenoise_256spp:\n"
    ".incbin \"" RT_STR(RT_DATA_DIR) "/bluenoise_256spp.u8\"\n"
    ".size rt_bluenoise_256spp, 327680\n"
    ".global rt_dither_rgb1_256\n"
    ".type rt_dither_rgb1_256, @object\n"
    ".balign 64\n"
    "rt_dither_rgb1_256:\n"
    ".incbin \"" RT_STR(RT_DATA_DIR) "/dither_rgb1_256.u8\"\n"
    ".size rt_dither_rgb1_256, 1572864\n"
    ".text\n");
