extern "C" const char* sdr_build_id(void) {
    static const char id[] = "SDR_BUILD_ID=c6839c98eccecf25";
    return id + 13;
}
