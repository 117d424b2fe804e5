# sourced by the A/B scripts that install abx/ (abv/) library variants over the in-tree
# libccsc.so: keep the tree's library and put it back on every exit path, so a
# later suite run in the same call never runs against a leftover variant
_lib=ccsc_code_iccv2017_amd/libccsc.so
_keep=$(mktemp /tmp/libccsc_keep.XXXXXX.so)
cp "$_lib" "$_keep"
trap 'cp "$_keep" "$_lib"; rm -f "$_keep"' EXIT
