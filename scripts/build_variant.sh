# Build a variant of the library for scripts/ab_libs.sh: bash scripts/build_variant.sh NAME "FLAGS"
set -e
cd "$(dirname "$0")/../asterisk-tiresias_amd"
make -s -j8 BUILD=abv/$1/build LIB=abv/$1/libtiresias_fp.so EXTRA="$2" abv/$1/libtiresias_fp.so
rm -rf abv/$1/build
