extern "C" const char* sdr_build_id(void) {
    static const char id[] = "SDR_BUILD_ID=1cc5cdd882dbc63e";
    return id + 13;
}
